# round 1 session 2: separable transform -- parity suite, smoke, bench line, kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r1s2b
mkdir -p $O/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 $O/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit=$rc"; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --variant none > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit=$rc"; cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --variant none --no-cpu-baseline > $O/prof/bench.json 2> $O/prof/bench.err
rc=$?; echo "rocprof exit=$rc"; [ $rc -eq 0 ] || exit $rc
head -12 $O/prof/bench_kernel_stats.csv | cut -c1-200
