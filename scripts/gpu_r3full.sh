# the whole -m gpu suite, smoke, then the default bench (round-3 confirmation runs)
set -o pipefail
out=gpurun_out/${1:-r3full}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $out/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac  # a fault, abort or time limit: nothing more on the GPU
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err
