set -o pipefail
out=gpurun_out/${1:-fsep}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fsep.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u scripts/bench_fsep.py 1024 128 > $out/bench_fsep.log 2>&1
