set -o pipefail
timeout -k 10 300 python scripts/debug_batch4.py 2>&1 | grep -v amdgpu.ids
