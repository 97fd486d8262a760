# round 2: device rand_func_int + ODE tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ode.py -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "PASS|FAIL|Error|assert" $O/tests.log | head -30; tail -3 $O/tests.log; exit $rc
