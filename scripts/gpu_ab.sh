# A/B timing of k_sdt_run builds (probe_sdt_ab.py), then the C4 parity tests on the default build
set -o pipefail
out=gpurun_out/${1:-ab}
mkdir -p $out
shift
timeout -k 10 300 python -u scripts/probe_sdt_ab.py 4096 "$@" > $out/ab.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -x -q --timeout 300 --timeout-method thread > $out/c4.log 2>&1
