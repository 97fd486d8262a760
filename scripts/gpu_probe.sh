set -o pipefail
out=gpurun_out/${1:-probe}
mkdir -p $out
export FS_LIB=${2:-libmioc_stamps.so}
timeout -k 10 120 python -u scripts/probe_fsep_phases.py 16 1 > $out/phases.log 2>&1 && \
timeout -k 10 120 python -u scripts/probe_fsep_phases.py 16 2 >> $out/phases.log 2>&1
