# one PMC pass (COUNTER = FETCH_SIZE or WRITE_SIZE) over the C4 headline alone; its own gpurun call (rocprofv3 7.2
# segfaults in exit() after writing its output, profiles/round3_profiler_exit_sigsegv.txt)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_c4}
C=${2:-FETCH_SIZE}
mkdir -p $O
A="--variant none --batch-config none --pinf-batch-config none --heat-restarts 0 --batch-total 0 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc $C -d $O/$C -o pmc --output-format csv -- python3 bench.py $A > $O/$C.log 2>&1
echo "$C exit=$?"; find $O -name "*counter_collection.csv"; exit 0
