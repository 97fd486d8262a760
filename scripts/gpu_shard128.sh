# what each rank of the 8-GPU strong-scaling batch line runs: 128 of the 1024 C5 restarts on one GPU
set -o pipefail
out=gpurun_out/${1:-shard128}
mkdir -p $out
timeout -k 10 600 python -u bench.py --variant none --pinf-batch-config none --heat-restarts 0 --batch-size 128 --batch-total 128 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
