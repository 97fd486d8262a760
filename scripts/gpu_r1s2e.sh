set -o pipefail
O=gpurun_out/r1s2e
mkdir -p $O
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -15 $O/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/probe_sdt_variants.py 4096 $PWD/$L/libmioc.so > $O/variants.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/variants.txt; exit $rc
