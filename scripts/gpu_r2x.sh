# round 2: p=Inf batch (small-L prep, banded walk): parity + throughput probe with and without R checkpoints
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "pinf or C1 or C2 or C3 or random or walk or golden or trm" > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for ck in 1; do
for c in C2 C3; do
PINF_CKPT=$ck timeout -k 10 300 python -u scripts/probe_pinf_batch.py $c 1 1024 > $O/$c.$ck.log 2>&1
rc=$?; grep -v amdgpu.ids $O/$c.$ck.log; [ $rc -eq 0 ] || exit $rc
done
done
