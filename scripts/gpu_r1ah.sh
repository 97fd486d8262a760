set -o pipefail
timeout -k 10 300 python scripts/probe_stamps.py 64 2>&1 | grep -v amdgpu.ids
