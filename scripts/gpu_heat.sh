# heat gradient line: smoke, bench line, kernel-trace stats (one GPU call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/heat
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python3 bench.py --config C2 --variant none --batch-config none --pinf-batch-config none > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o heat --output-format csv -- python3 bench.py --config C2 --variant none --batch-config none --pinf-batch-config none --no-cpu-baseline > $O/prof.log 2>&1
echo "prof exit=$?"
