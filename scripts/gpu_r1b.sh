set -o pipefail
mkdir -p gpurun_out/prof_r1b
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=500 -p no:cacheprovider > gpurun_out/gpu_tests_r1b.log 2>&1
echo "tests exit=$?" >> gpurun_out/gpu_tests_r1b.log
tail -5 gpurun_out/gpu_tests_r1b.log
timeout -k 10 420 python bench.py > gpurun_out/bench_r1b.json 2> gpurun_out/bench_r1b.err
rc=$?
echo "bench exit=$rc"; cat gpurun_out/bench_r1b.json; tail -5 gpurun_out/bench_r1b.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_r1b/bench.json 2> gpurun_out/prof_r1b/bench.err
echo "rocprof exit=$?"
find gpurun_out/prof_r1b -name "*stats*" | head
