set -o pipefail
O=gpurun_out/r1s2g
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_nt.py 256 1024 4096 16384 > $O/nt.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/nt.txt; exit $rc
