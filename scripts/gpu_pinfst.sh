set -o pipefail
out=gpurun_out/${1:-pinfst}
mkdir -p $out
timeout -k 10 120 python -u scripts/probe_pinf_stamps.py 16384 > $out/st.log 2>&1
