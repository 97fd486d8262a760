# k_fsep2 write-phase clocks at 128 restarts, S = 2 (libmioc_stamps_w.so: MIOC_STAMPS_WRITE)
set -o pipefail
out=gpurun_out/${1:-fsph2}
mkdir -p $out
FS_LIB=libmioc_stamps_w.so FS_WPB=8 timeout -k 10 120 python -u scripts/probe_fsep_phases.py 128 2 > $out/w4.log 2>&1
