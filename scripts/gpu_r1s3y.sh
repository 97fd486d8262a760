set -o pipefail
O=gpurun_out/r1s3y
mkdir -p $O
timeout -k 10 200 python scripts/probe_sdt_batch.py 4096 1 3 > $O/k1.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k1.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_sdt_batch.py 4096 2 3 > $O/k2.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k2.txt; exit $rc
