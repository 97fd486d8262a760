# round 2: fused small-state batch DP -- parity (batch + existing suites) and a C5 batch bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/batch.log 2>&1
rc=$?; echo "batch tests exit=$rc"; tail -15 $O/batch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C5 --batch 1024 --steps 3 --warmup 1 --variant none --no-cpu-baseline > $O/c5.json 2> $O/c5.err
rc=$?; echo "c5 exit=$rc"; cat $O/c5.json; tail -3 $O/c5.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 $O/tests.log; exit $rc
