set -o pipefail
O=gpurun_out/r2p
mkdir -p $O
L=$PWD/mixed-integer-optimal-control---algorithm-tools_amd/lib
for v in "" _v1; do
for K in 1 2; do
MIOC_LIB=$L/libmioc$v.so timeout -k 10 300 python scripts/probe_sdt_batch.py 8192 $K 2 > $O/k$K$v.txt 2>&1
rc=$?; echo "lib [$v]"; grep -v amdgpu.ids $O/k$K$v.txt | head -1; [ $rc -eq 0 ] || exit $rc
done
done
