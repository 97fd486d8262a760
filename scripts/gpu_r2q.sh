set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2q
mkdir -p $O
timeout -k 10 300 python scripts/probe_sdt_batch.py 8192 1 2 > $O/k1.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k1.txt | head -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_batch.py 4096 2 1 > $O/k2.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; exit $rc
