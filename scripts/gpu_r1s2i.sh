set -o pipefail
O=gpurun_out/r1s2i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 $O/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/probe_sdt_nt.py 4096 > $O/nt.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/nt.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_timeline.py 1024 > $O/timeline.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/timeline.txt; exit $rc
