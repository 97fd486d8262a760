set -o pipefail
O=gpurun_out/r1s3c
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_timeline.py 1024 > $O/timeline.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/timeline.txt; exit $rc
