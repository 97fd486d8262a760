set -o pipefail
O=gpurun_out/r1s2k
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_nt.py 4096 > $O/nt.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/nt.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_timeline.py 1024 > $O/timeline.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/timeline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_stamps.py 256 1 > $O/stamps_p.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps_p.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_stamps.py 256 0 > $O/stamps_s.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps_s.txt; exit $rc
