# round 2: C4-shape parity on k_sdt_run vs the oracle (fixture + tie-heavy + chunked rows), 8^3 off-grid u_old
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4.py "tests/test_gpu_parity.py::test_pyramid_vs_oracle_512_levels" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $O/c4.log 2>&1
rc=$?; echo "c4 tests exit=$rc"; grep -E "PASS|FAIL|Error|passed|failed" $O/c4.log | tail -40; exit $rc
