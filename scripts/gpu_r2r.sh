set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; exit $rc
