# round 2: p=Inf batch throughput probe (C2 / C3 shapes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 300 python -u scripts/probe_pinf_batch.py C2 1 64 256 1024 > $O/c2.log 2>&1
rc=$?; cat $O/c2.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_pinf_batch.py C3 1 64 256 1024 > $O/c3.log 2>&1
rc=$?; cat $O/c3.log | grep -v amdgpu.ids; exit $rc
