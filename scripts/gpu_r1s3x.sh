set -o pipefail
O=gpurun_out/r1s3x
mkdir -p $O
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
for r in 1 2; do
MIOC_LIB=$PWD/$L/libmioc_base.so timeout -k 10 200 python scripts/probe_sdt_rep.py 8192 6 > $O/base$r.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/base$r.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_sdt_rep.py 8192 6 > $O/new$r.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/new$r.txt; [ $rc -eq 0 ] || exit $rc
done
