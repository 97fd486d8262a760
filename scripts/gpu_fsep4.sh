# k_fsep2 four lanes per row (row segments) vs two: C5 timings at 128 and 1024 restarts, the fsep parity tests,
# then the k_sdt_run split-chain A/B
set -o pipefail
out=gpurun_out/${1:-fsep4}
mkdir -p $out
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
MIOC_LIB=$L/libmioc_l2.so timeout -k 10 200 python -u scripts/bench_fsep.py 128 > $out/l2.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/bench_fsep.py 128 1024 > $out/l4.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fsep.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/probe_sdt_ab.py 4096 $L/libmioc_split.so $L/libmioc.so > $out/ab.log 2>&1
