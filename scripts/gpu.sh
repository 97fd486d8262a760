# One runner for every GPU step of this repository, run on the GPU box by gpurun:
#     gpurun --timeout 1200 -- bash scripts/gpu.sh <out> <step> [<step> ...]
# Output goes to gpurun_out/<out>/ (one log per step).  Steps run in order, each under its own time limit; the first
# step that fails, times out or dies ends the call (no GPU step after a fault).  Arguments inside a step are separated
# by commas (a step is one shell word).
#   tests              pytest -m gpu over tests/ (tests:f1.py,f2.py[::name]: only those files / tests)
#   bench[:args]       python bench.py args                       -> bench.json
#   smoke              __graft_entry__.smoke()
#   prof[:args]        rocprofv3 --kernel-trace --stats over bench.py args   -> prof/ (kernel_stats.csv)
#   pmc:c1+c2[:args]   ONE rocprofv3 --pmc pass (counters joined by +) over bench.py args -> pmc_<c1>/
#   py:script[,args]   python scripts/<script> args (probes, A/B harnesses)
#   exe:path[,args]    a binary built in this container (e.g. scripts/ubench/pass_occ)
#   with:VAR=value     export VAR for the steps that follow (e.g. with:MIOC_LIB=<a variant build>)
#   pyprof:script[,args]  rocprofv3 --kernel-trace --stats over python scripts/<script> args -> pyprof/
#   pypmc:c1+c2:script[,args]  ONE rocprofv3 --pmc pass over python scripts/<script> args -> pypmc<n>/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?usage: gpu.sh <out> <step>...}
shift
mkdir -p "$O"
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=""
  [ "$kind" != "$step" ] && rest=${step#*:}
  args=${rest//,/ }
  log="$O/$n-$kind.log"
  echo "== step $n: $step"
  case "$kind" in
    tests)
      sel="tests"
      [ -n "$rest" ] && sel=$(for f in $args; do echo -n "tests/$f "; done)
      timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 240 --timeout-method thread \
        -p no:cacheprovider > "$log" 2>&1
      rc=$?; tail -3 "$log" ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > "$O/bench$n.json" 2> "$log"
      rc=$?; cat "$O/bench$n.json"; tail -2 "$log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof$n" -o prof --output-format csv \
        -- python3 bench.py $args > "$O/bench_prof$n.json" 2> "$log"
      rc=$?; cat "$O/bench_prof$n.json"; find "$O/prof$n" -name "*kernel_stats.csv" ;;
    pmc)
      ctr=${rest%%:*}
      bargs=""
      [ "$ctr" != "$rest" ] && bargs=${rest#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//+/ } -d "$O/pmc$n" -o pmc --output-format csv \
        -- python3 bench.py ${bargs//,/ } > "$log" 2>&1
      rc=$?; find "$O/pmc$n" -name "*counter_collection.csv" ;;
    py)
      timeout -k 10 600 python -u scripts/$args > "$log" 2>&1
      rc=$?; tail -40 "$log" ;;
    pypmc)
      ctr=${rest%%:*}
      sargs=${rest#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//+/ } -d "$O/pypmc$n" -o pmc --output-format csv \
        -- python3 scripts/${sargs//,/ } > "$log" 2>&1
      rc=$?; tail -3 "$log"; find "$O/pypmc$n" -name "*counter_collection.csv" ;;
    pyprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/pyprof$n" -o prof --output-format csv \
        -- python3 scripts/$args > "$log" 2>&1
      rc=$?; tail -5 "$log"; find "$O/pyprof$n" -name "*kernel_stats.csv" ;;
    with)
      export "$rest"; echo "exported $rest"; rc=0 ;;
    exe)
      timeout -k 10 300 $args > "$log" 2>&1
      rc=$?; tail -40 "$log" ;;
    *)
      echo "unknown step $kind"; exit 2 ;;
  esac
  echo "== step $n exit=$rc"
  [ $rc -eq 0 ] || exit $rc
done
