set -o pipefail
mkdir -p gpurun_out/r1ad
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "batch" > gpurun_out/r1ad/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r1ad/tests.log; exit $rc
