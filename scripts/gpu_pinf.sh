# p=Inf segmented walk: its parity tests, the p=Inf parity suite, then the C4 p=Inf bench line
set -o pipefail
out=gpurun_out/${1:-pinf}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pinf_walk.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u bench.py --p inf --variant none --batch-config none --heat-restarts 0 --pinf-batch-config none --no-cpu-baseline > $out/bench_pinf.json 2> $out/bench_pinf.err
