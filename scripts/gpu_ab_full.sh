# A/B timing of k_sdt_run builds, the load-issue timeline, then the whole -m gpu suite on the default build
set -o pipefail
out=gpurun_out/${1:-abf}
mkdir -p $out
shift
timeout -k 10 300 python -u scripts/probe_sdt_ab.py 4096 "$@" > $out/ab.log 2>&1 || exit $?
timeout -k 10 180 python -u scripts/probe_sdt_timeline.py 8192 64 $out/tl.npy > $out/timeline.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
