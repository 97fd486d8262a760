set -o pipefail
mkdir -p gpurun_out/pmc_r1g
export TMPDIR=/tmp
timeout -k 10 300 python scripts/probe_pyr.py 512 > gpurun_out/probe_r1g.txt 2>&1; echo "probe exit=$?"; cat gpurun_out/probe_r1g.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout=500 -p no:cacheprovider -k "pyramid or golden or c4" > gpurun_out/gpu_tests_r1g.log 2>&1; echo "tests exit=$?"; tail -3 gpurun_out/gpu_tests_r1g.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY -d gpurun_out/pmc_r1g -o pmc1 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/pmc_r1g/p1.txt 2>&1; echo "pmc1 exit=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 -d gpurun_out/pmc_r1g -o pmc2 --output-format csv -- python3 scripts/probe_pyr.py 64 > gpurun_out/pmc_r1g/p2.txt 2>&1; echo "pmc2 exit=$?"
