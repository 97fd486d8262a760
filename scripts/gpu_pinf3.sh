set -o pipefail
out=gpurun_out/${1:-pinf3}
mkdir -p $out
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
timeout -k 10 300 python -u scripts/probe_pinf_c4.py 65536 $L/libmioc_g2.so $L/libmioc.so $L/libmioc_g2.so $L/libmioc.so > $out/ab.log 2>&1
