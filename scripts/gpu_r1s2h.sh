set -o pipefail
O=gpurun_out/r1s2h
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_nt.py 4096 > $O/nt.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/nt.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_timeline.py 1024 > $O/timeline.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/timeline.txt; exit $rc
