# round-end check on one box: the GPU suite, the default bench line, smoke, then a kernel-trace profile of the
# default bench (its k_* averages must agree with the bench's HIP events)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
bash scripts/gpu_full.sh ${1:-final} || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o ks --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof.json 2> $O/prof.err
echo "prof exit=$?"; find $O/prof -name "*stats.csv"
