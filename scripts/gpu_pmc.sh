# one rocprofv3 PMC pass (its own gpurun call: rocprofv3 7.2 segfaults in exit() after writing its output)
# usage: bash scripts/gpu_pmc.sh OUTDIR COUNTER [bench.py args ...]
#   e.g. bash scripts/gpu_pmc.sh r2h_fetch FETCH_SIZE --config C2 --variant none --batch-config none \
#        --pinf-batch-config none --steps 1 --warmup 0 --no-cpu-baseline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
C=$2
shift 2
mkdir -p $O
timeout -s KILL 400 rocprofv3 --pmc $C -d $O/pmc -o pmc --output-format csv -- python3 bench.py "$@" > $O/pmc.log 2>&1
rc=$?; echo "$C exit=$rc"; find $O -name "*counter_collection.csv"; exit 0
