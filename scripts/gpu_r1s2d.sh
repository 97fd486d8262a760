set -o pipefail
O=gpurun_out/r1s2d
mkdir -p $O
L=mixed-integer-optimal-control---algorithm-tools_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "separable or 512 or c4_scale or golden" > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -5 $O/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python scripts/probe_sdt_variants.py 4096 $PWD/$L/libmioc.so $PWD/$L/libmioc_sc1.so > $O/variants.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/variants.txt; exit $rc
