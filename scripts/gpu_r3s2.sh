# session-2 check: k_sdt_run A/B at nt = 4096, then the round-end sequence (GPU suite, bench, smoke, rocprof trace)
set -o pipefail
O=gpurun_out/${1:-r3s2}
mkdir -p $O
timeout -k 10 300 python -u scripts/probe_sdt_ab.py 4096 mixed-integer-optimal-control---algorithm-tools_amd/lib/libmioc.so > $O/ab.log 2>&1 || exit $?
bash scripts/gpu_final.sh ${1:-r3s2}
