# k_fsep2 phase clocks at 128 restarts, S = 2: four lanes per row (libmioc_stamps.so) vs two (libmioc_stamps_l2.so)
set -o pipefail
out=gpurun_out/${1:-fsph}
mkdir -p $out
FS_WPB=8 timeout -k 10 120 python -u scripts/probe_fsep_phases.py 128 2 > $out/l4.log 2>&1 || exit $?
FS_LIB=libmioc_stamps_l2.so FS_WPB=4 timeout -k 10 120 python -u scripts/probe_fsep_phases.py 128 2 > $out/l2.log 2>&1
