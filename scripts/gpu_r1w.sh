set -o pipefail
mkdir -p gpurun_out/r1w
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider -k "pyramid or golden or c4 or random" > gpurun_out/r1w/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r1w/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_pyr.py 2048 2>&1 | grep -v amdgpu.ids
