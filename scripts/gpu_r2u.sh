# round 2 PMC pass 2 (its own call: rocprofv3 7.2 segfaults in exit() after writing its output, see profiles/README.md)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2u
mkdir -p $O
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1
rc=$?; echo "write exit=$rc"; exit $rc
