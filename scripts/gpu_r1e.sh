set -o pipefail
mkdir -p gpurun_out/pmc_r1e
export TMPDIR=/tmp
timeout -k 10 300 python scripts/probe_pyr.py 512 > gpurun_out/probe_r1e.txt 2>&1; echo "probe exit=$?"; cat gpurun_out/probe_r1e.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM -d gpurun_out/pmc_r1e -o pmc1 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/pmc_r1e/p1.txt 2>&1; echo "pmc1 exit=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MIN_MAX_F64 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_r1e -o pmc2 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/pmc_r1e/p2.txt 2>&1; echo "pmc2 exit=$?"
ls gpurun_out/pmc_r1e
