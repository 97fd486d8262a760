# round 2: k_sdt_run with the drain deferred across interleaved subproblems: parity, then per-step time K=1/2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "c4 or separable or golden" > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for K in 1 2; do
timeout -k 10 300 python -u scripts/probe_sdt_batch.py 8192 $K 2 > $O/k$K.log 2>&1
rc=$?; grep -v amdgpu.ids $O/k$K.log | head -3; [ $rc -eq 0 ] || exit $rc
done
