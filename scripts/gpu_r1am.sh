set -o pipefail
O=gpurun_out/r1am
mkdir -p $O
timeout -k 10 300 python scripts/probe_pinf_stamps.py 65536 > $O/pinf_stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/pinf_stamps.txt; exit $rc
