set -o pipefail
timeout -k 10 300 python scripts/probe_pyr.py 512 2>&1 | grep -v amdgpu.ids
