# round 2 profiles: kernel-trace stats of the default bench, then FETCH_SIZE / WRITE_SIZE passes (separate runs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2s
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/ks -o ks -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err
rc=$?; echo "stats exit=$rc"; cat $O/bench_prof.json; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1
rc=$?; echo "fetch exit=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1
rc=$?; echo "write exit=$rc"; find $O -name "*.csv" | head -20; exit $rc
