set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "pyramid or golden or c4" > gpurun_out/r1i_tests.log 2>&1 && tail -3 gpurun_out/r1i_tests.log &&
timeout -k 10 300 python scripts/probe_pyr.py 512 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 300 python scripts/probe_stamps.py 64 2>&1 | grep -v amdgpu.ids
