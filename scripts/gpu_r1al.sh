# round 1: parity after the branch-free p=Inf walk; p=Inf walk timing; k_pinf_recur phase stamps
set -o pipefail
O=gpurun_out/r1al
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x --timeout=600 -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_walk.py 65536 inf > $O/walk_inf.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/walk_inf.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_pinf_stamps.py 65536 > $O/pinf_stamps.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/pinf_stamps.txt; exit $rc
