# C4 parity on the persistent kernel, the C4 bench line, the kernel timeline (round 3 iteration script)
set -o pipefail
out=gpurun_out/${1:-r3b}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -x -q --timeout 240 --timeout-method thread > $out/c4.log 2>&1
echo "c4 rc=$?" >> $out/c4.log
timeout -k 10 200 python -u bench.py --variant none --batch-config none --pinf-batch-config none --heat-restarts 0 --no-cpu-baseline --steps 2 --warmup 1 > $out/bench.json 2> $out/bench.err
echo "bench rc=$?" >> $out/bench.err
timeout -k 10 200 python -u scripts/probe_sdt_timeline.py 8192 64 $out/tl.npy > $out/tl.txt 2>&1
