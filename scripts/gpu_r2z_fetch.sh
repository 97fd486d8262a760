# round 2 PMC pass over the C2 p=Inf batch line alone (its own call: rocprofv3 segfaults in exit() after writing)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2z
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 bench.py --config C2 --batch 1024 --variant none --batch-config none --pinf-batch-config none --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1
rc=$?; echo "fetch exit=$rc"; exit $rc
