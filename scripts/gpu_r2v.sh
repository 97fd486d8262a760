# round 2: TRM quantities (pred / TV_p / decide) on the device + smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_trm.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit=$rc"; tail -2 $O/smoke.log; exit $rc
