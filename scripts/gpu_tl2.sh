set -o pipefail
out=gpurun_out/${1:-tl2}
mkdir -p $out
timeout -k 10 180 python -u scripts/probe_sdt_timeline.py 8192 64 $out/tl.npy > $out/timeline.log 2>&1
