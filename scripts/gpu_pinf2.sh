# k_pinf_recur class split (four lanes per row pair) vs one lane: C4 p=Inf A/B, then the p=Inf parity tests
set -o pipefail
out=gpurun_out/${1:-pinf2}
mkdir -p $out
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
timeout -k 10 300 python -u scripts/probe_pinf_c4.py 65536 $L/libmioc_pinf1.so $L/libmioc.so > $out/ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_pinf_walk.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
