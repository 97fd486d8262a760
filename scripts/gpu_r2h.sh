set -o pipefail
O=gpurun_out/r2h
mkdir -p $O
L=$PWD/mixed-integer-optimal-control---algorithm-tools_amd/lib
for v in _v1 _v2; do
  for a in 6 5; do
  MIOC_LIB=$L/libmioc$v.so timeout -k 10 120 python scripts/probe_fused.py 1024 plain $a > $O/f$v$a.txt 2>&1
  rc=$?; echo "variant [$v] algo $a (no U stores)"; grep -v amdgpu.ids $O/f$v$a.txt | tail -2; [ $rc -eq 0 ] || exit $rc
  done
done
