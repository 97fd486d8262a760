set -o pipefail
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 200 python scripts/probe_fused.py 1024 stamps > $O/stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_fused.py 1024 > $O/plain.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/plain.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_fused.py 256 > $O/k256.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k256.txt; exit $rc
