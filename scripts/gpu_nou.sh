set -o pipefail
out=gpurun_out/${1:-nou}
mkdir -p $out
MIOC_LIB=mixed-integer-optimal-control---algorithm-tools_amd/lib/libmioc_nou.so timeout -k 10 200 python -u scripts/bench_fsep.py 128 1024 > $out/nou.log 2>&1
