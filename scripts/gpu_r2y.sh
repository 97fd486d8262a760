# round 2: default bench (now with the C2 p=Inf batch line)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2y
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench exit=$rc"; cat $O/bench.json; tail -3 $O/bench.err; exit $rc
