# C4 parity on the persistent kernel, the C4 bench line, the kernel timeline, and A/B variants (round-3 iteration)
# usage: bash scripts/gpu_r3b.sh OUTDIR [variant ...]   (variant = NAME of lib/libmioc_NAME.so)
set -o pipefail
out=gpurun_out/${1:-r3b}
shift
mkdir -p $out
LIB=mixed-integer-optimal-control---algorithm-tools_amd/lib
bench() {
  timeout -k 10 200 python -u bench.py --variant none --batch-config none --pinf-batch-config none --heat-restarts 0 \
    --no-cpu-baseline --steps 2 --warmup 1 > $out/bench_$1.json 2> $out/bench_$1.err
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -x -q --timeout 240 --timeout-method thread > $out/c4.log 2>&1 || exit 1
bench base || exit 1
for v in "$@"; do
  MIOC_LIB=$LIB/libmioc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_c4.py -x -q -k fixture --timeout 240 \
    --timeout-method thread > $out/c4_$v.log 2>&1 || exit 1
  MIOC_LIB=$LIB/libmioc_$v.so bench $v || exit 1
done
timeout -k 10 200 python -u scripts/probe_sdt_timeline.py 8192 64 $out/tl.npy > $out/tl.txt 2>&1
