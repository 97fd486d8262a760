set -o pipefail
O=gpurun_out/r1s2c
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_stamps.py 64 > $O/sdt_stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/sdt_stamps.txt; exit $rc
