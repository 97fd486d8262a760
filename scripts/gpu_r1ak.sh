# round 1: parity suite after the run-ahead walks + walk timings at C4 scale (p=1 pyramid, p=Inf)
set -o pipefail
O=gpurun_out/r1ak
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_walk.py 65536 inf > $O/walk_inf.txt 2>&1
rc=$?; cat $O/walk_inf.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_walk.py 65536 1 > $O/walk_p1.txt 2>&1
rc=$?; cat $O/walk_p1.txt | grep -v amdgpu.ids; exit $rc
