set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/batch.log 2>&1
rc=$?; echo "batch tests exit=$rc"; tail -4 $O/batch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/probe_fused.py 1024 plain 6 > $O/fsep.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/fsep.txt | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/probe_fused.py 256 stamps 6 > $O/st.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/st.txt | tail -10; exit $rc
timeout -k 10 120 python scripts/probe_fused.py 256 stamps 6 > $O/st2.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/st2.txt | tail -5; exit $rc
