# round 2: mioc_batch_multi + device ODE gradient producer
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ode.py tests/test_gpu_batch.py -x -v -s --timeout 240 --timeout-method thread -p no:cacheprovider -k "ode or multi or trust or batch" > $O/tests.log 2>&1
rc=$?; echo "tests exit=$rc"; grep -E "bit-identical|PASS|FAIL|Error|error" $O/tests.log | head -30; tail -3 $O/tests.log; exit $rc
