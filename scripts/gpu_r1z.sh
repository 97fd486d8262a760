set -o pipefail
for lib in libmioc_prev.so libmioc.so libmioc_stamps.so; do
  echo "== $lib"
  MIOC_LIB=$PWD/mixed-integer-optimal-control---algorithm-tools_amd/lib/$lib timeout -k 10 300 python scripts/probe_pyr.py 512 2>&1 | grep -v amdgpu.ids || exit 1
done
