set -o pipefail
O=gpurun_out/r2g
mkdir -p $O
for K in 256 512 1024; do
timeout -k 10 120 python scripts/probe_fused.py $K plain 6 > $O/k$K.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k$K.txt | tail -2; [ $rc -eq 0 ] || exit $rc
done
