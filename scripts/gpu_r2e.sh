set -o pipefail
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 200 python scripts/probe_fused.py 1024 stamps 6 > $O/stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_fused.py 256 plain 6 > $O/k256.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps256.txt; exit $rc
