# the error-code / validation tests, then the C4 + C5 batch bench lines
set -o pipefail
out=gpurun_out/${1:-val}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --variant none --pinf-batch-config none --heat-restarts 0 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
