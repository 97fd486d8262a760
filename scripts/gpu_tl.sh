# phase stamps (libmioc_stamps.so) and the pipeline timeline (libmioc_stamps_tl.so) of k_sdt_run at C4 shape
set -o pipefail
out=gpurun_out/${1:-tl}
mkdir -p $out
timeout -k 10 120 python -u scripts/probe_sdt_stamps.py 512 1 > $out/stamps.log 2>&1 || exit $?
timeout -k 10 180 python -u scripts/probe_sdt_timeline.py 8192 64 > $out/timeline.log 2>&1
