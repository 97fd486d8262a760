"""bench.py's multi-rank launcher on the CPU (gloo): `bench.py --gpus 2` starts two ranks itself, shards each
step's global batch, gathers the controls (uint16 level ranks) and Φ* to rank 0 and reports n_gpus = 2, with
results identical to one rank solving the whole batch.  The per-rank solver here is the CPU oracle (test double);
on GPUs the same launcher / shard / gather code drives libmioc over RCCL."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, batch, total=0):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--solver", "oracle", "--backend",
           "gloo", "--config", "C5", "--nt", "10", "--batch", str(batch), "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--total", str(total)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_launcher_world2_matches_world1():
    two = _bench(2, 2)
    one = _bench(1, 4)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["scaling"] == "weak"
    # the same global batch per step (world x batch = 4 restarts): identical controls and Φ*
    assert two["checksum"] == one["checksum"]
    assert two["value"] > 0 and one["value"] > 0


def test_launcher_strong_scaling_world2_matches_world1():
    """Strong scaling (`--total`, the mode of bench.py's batch_strong line): a fixed global batch per step split
    over the ranks -- 5 restarts as 3 + 2 on two ranks -- gives the same controls and Φ* as one rank solving all 5."""
    two = _bench(2, 1, total=5)
    one = _bench(1, 1, total=5)
    assert two["scaling"] == "strong" and one["scaling"] == "strong"
    assert two["checksum"] == one["checksum"]
    weak = _bench(1, 5)
    assert weak["checksum"] == one["checksum"] and weak["scaling"] == "weak"
