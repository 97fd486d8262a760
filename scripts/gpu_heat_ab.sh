# A/B of k_heat_run builds: the default library against variants under mixed-integer-optimal-control---algorithm-tools_amd/lib/var/
set -o pipefail
O=gpurun_out/heat_ab
mkdir -p $O
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
for v in $L/libmioc.so $L/var/*.so; do
  MIOC_LIB=$v timeout -k 10 120 python3 scripts/probe_heat.py 4096 >> $O/ab.log 2>&1 || { echo "fail $v"; exit 1; }
done
grep -v amdgpu.ids $O/ab.log
