# round 2: K=2 interleaved persistent separable transform -- memory, timing, parity
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 60 python -c "import torch; f,t=torch.cuda.mem_get_info(); print('free GB', f/1e9, 'total GB', t/1e9)" 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python scripts/probe_sdt_batch.py 8192 1 2 > $O/k1.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k1.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_batch.py 8192 2 2 > $O/k2.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/k2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/c4.log 2>&1
rc=$?; echo "c4 tests exit=$rc"; tail -3 $O/c4.log; exit $rc
