set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=500 -p no:cacheprovider > gpurun_out/gpu_tests_r1c.log 2>&1
echo "tests exit=$?" >> gpurun_out/gpu_tests_r1c.log
tail -4 gpurun_out/gpu_tests_r1c.log
timeout -k 10 300 python bench.py --p inf --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_pinf_r1c.json 2> gpurun_out/bench_pinf_r1c.err
echo "bench exit=$?"; cat gpurun_out/bench_pinf_r1c.json; tail -3 gpurun_out/bench_pinf_r1c.err
