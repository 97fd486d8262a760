# one PMC pass: VALU instructions and waves of the C4 kernels (nt truncated to 8192), its own gpurun call
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_valu}
mkdir -p $O
A="--variant none --batch-config none --pinf-batch-config none --heat-restarts 0 --batch-total 0 --steps 1 --warmup 0 --no-cpu-baseline --nt 8192"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/pmc -o pmc --output-format csv -- python3 bench.py $A > $O/pmc.log 2>&1
echo "exit=$?"; find $O -name "*counter_collection.csv"; exit 0
