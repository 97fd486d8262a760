# round 2 PMC passes (separate runs): FETCH_SIZE, WRITE_SIZE over one bench step of every line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2t
mkdir -p $O
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1
rc=$?; echo "fetch exit=$rc"; tail -2 $O/fetch.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1
rc=$?; echo "write exit=$rc"; find $O -name "*.csv"; exit $rc
