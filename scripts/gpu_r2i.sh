set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 120 python scripts/probe_fused.py 256 stamps 6 > $O/st.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/st.txt | tail -12; exit $rc
