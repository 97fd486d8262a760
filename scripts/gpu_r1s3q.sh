set -o pipefail
O=gpurun_out/r1s3q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "512_levels or c4_scale or separable or sdt" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_nt.py 4096 > $O/nt.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/nt.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_timeline.py 1024 > $O/timeline.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/timeline.txt | head -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_stamps.py 256 1 > $O/stamps_p.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps_p.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_sdt_stamps.py 256 0 > $O/stamps_s.txt 2>&1
rc=$?; grep -v amdgpu.ids $O/stamps_s.txt; exit $rc
