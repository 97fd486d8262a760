set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
L=$PWD/mixed-integer-optimal-control---algorithm-tools_amd/lib
for v in "" _v1 _v2 _v3; do
  MIOC_LIB=$L/libmioc$v.so timeout -k 10 120 python scripts/probe_fused.py 1024 plain 6 > $O/fsep$v.txt 2>&1
  rc=$?; echo "variant [$v]"; grep -v amdgpu.ids $O/fsep$v.txt | tail -2; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 120 python scripts/probe_fused.py 1024 plain 5 > $O/brute.txt 2>&1
rc=$?; echo "brute force"; grep -v amdgpu.ids $O/brute.txt | tail -2; exit $rc
