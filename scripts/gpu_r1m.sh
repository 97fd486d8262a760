set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1m
timeout -k 10 300 python scripts/probe_stamps.py 64 2>&1 | grep -v amdgpu.ids &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r1m -o pmc1 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/r1m/p1.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d gpurun_out/r1m -o pmc2 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/r1m/p2.txt 2>&1
echo "exit=$?"
