set -o pipefail
mkdir -p gpurun_out/r1ac
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/r1ac/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r1ac/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --p inf --steps 3 --warmup 1 --no-cpu-baseline --variant none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['backtrack_ms'])" &&
timeout -k 10 300 python scripts/probe_pyr.py 512 2>&1 | grep -v amdgpu.ids
