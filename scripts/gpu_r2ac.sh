set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2ac
mkdir -p $O
timeout -k 10 200 python -u scripts/probe_trm_batch.py 1 > $O/probe.log 2>&1
rc=$?; grep -v amdgpu.ids $O/probe.log | tail -40; exit $rc
