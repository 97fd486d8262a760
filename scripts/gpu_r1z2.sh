set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1z2
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r1z2 -o tr --output-format csv -- python3 scripts/probe_pyr.py 512 > gpurun_out/r1z2/p.txt 2>&1
echo "exit=$?"
