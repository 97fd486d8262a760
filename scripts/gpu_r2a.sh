# round 2 baseline: GPU parity suite, C4 bench (short), C5 batch on the pre-round-2 path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --variant none --no-cpu-baseline > $O/c4.json 2> $O/c4.err
rc=$?; echo "c4 exit=$rc"; cat $O/c4.json; tail -3 $O/c4.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --batch 1024 --steps 2 --warmup 1 --variant none --no-cpu-baseline > $O/c5.json 2> $O/c5.err
rc=$?; echo "c5 exit=$rc"; cat $O/c5.json; tail -3 $O/c5.err; exit $rc
