set -o pipefail
mkdir -p gpurun_out/prof_r1d
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > gpurun_out/gpu_tests_r1d.log 2>&1
echo "tests exit=$?" >> gpurun_out/gpu_tests_r1d.log
tail -4 gpurun_out/gpu_tests_r1d.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r1d.json 2> gpurun_out/bench_r1d.err
rc=$?; echo "bench exit=$rc"; cat gpurun_out/bench_r1d.json; tail -3 gpurun_out/bench_r1d.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1d -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_r1d/bench.json 2> gpurun_out/prof_r1d/bench.err
echo "rocprof exit=$?"
