set -o pipefail
mkdir -p gpurun_out/r1y
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/r1y/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r1y/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_pyr.py 512 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 300 python scripts/probe_stamps.py 64 2>&1 | grep -v amdgpu.ids | tail -4
