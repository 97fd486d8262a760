# round 1: full GPU parity suite, bench line, rocprof kernel stats of the bench command, HBM PMC passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r1s3z
mkdir -p $O/prof $O/pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit=$rc"; cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py > $O/prof/bench.json 2> $O/prof/bench.err
rc=$?; echo "rocprof exit=$rc"; [ $rc -eq 0 ] || exit $rc
A="--steps 1 --warmup 0 --variant none --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o p1_fetch --output-format csv -- python3 bench.py $A > $O/pmc/p1_fetch.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o p1_write --output-format csv -- python3 bench.py $A > $O/pmc/p1_write.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o pinf_fetch --output-format csv -- python3 bench.py $A --p inf > $O/pmc/pinf_fetch.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc -o pinf_write --output-format csv -- python3 bench.py $A --p inf > $O/pmc/pinf_write.txt 2>&1
rc=$?; echo "pmc exit=$rc"; find $O/pmc -name "*.csv"
