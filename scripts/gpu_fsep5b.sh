# k_fsep2 with the inbox polled a step ahead: C5 timings at 128 and 1024 restarts, the fsep/batch parity tests
set -o pipefail
out=gpurun_out/${1:-fsep5b}
mkdir -p $out
timeout -k 10 200 python -u scripts/bench_fsep.py 128 1024 > $out/l4.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_fsep.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
