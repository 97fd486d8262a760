# round 2: fused separable DP (p=1, 2-D grids) -- batch parity, timing, full GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/batch.log 2>&1
rc=$?; echo "batch tests exit=$rc"; tail -22 $O/batch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe_fused.py 1024 plain 6 > $O/fsep.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/fsep.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 $O/tests.log; exit $rc
