# device-resident TRM control: the TRM_batch parity tests (ODE and heat), then the heat probe
set -o pipefail
out=gpurun_out/${1:-trm}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode.py tests/test_heat.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u scripts/probe_heat_trm.py 1024 17 500 10 > $out/probe.log 2>&1
