set -o pipefail
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 400 python scripts/probe_c4_tail.py 51 > $O/tail.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/tail.txt | tail -40; exit $rc
