"""The single-subproblem bench lines (bench.py single_C2 / single_C3: one subproblem per step, bellman + backtrack
through the device-tensor entry points, no host sync inside the timed loop), timed alone.
Usage: python scripts/probe_single.py [CFG] [steps]   (MIOC_LIB selects a library build)
Under rocprofv3 --kernel-trace the per-kernel durations and the gaps between them show where a step goes."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = CONFIGS[cfg_name]
lt = cfg.levels()
n = steps + 3
dfs, uos = [], []
for s in range(n):
    _, df, uo = make_inputs(cfg, k=s, nt=cfg.nt, levels=lt)
    dfs.append(torch.tensor(np.ascontiguousarray(df.T[None]), dtype=torch.float64, device="cuda"))
    uos.append(torch.tensor(np.ascontiguousarray(uo.T[None]), dtype=torch.float64, device="cuda"))
du = torch.empty_like(dfs[0])
dphi = torch.empty(1, dtype=torch.float64, device="cuda")
dst = torch.empty(1, dtype=torch.int32, device="cuda")
with native.Context(0) as ctx:
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    for s in range(3):
        ctx.bellman_batch_tensors(dfs[s], uos[s], cfg.B, cfg.dt)
        ctx.backtrack_batch_tensors(cfg.B, du, dphi, dst)
    ctx.synchronize()
    torch.cuda.synchronize()
    ctx.reset_stats()
    t0 = time.perf_counter()
    for s in range(3, n):
        ctx.bellman_batch_tensors(dfs[s], uos[s], cfg.B, cfg.dt)
        ctx.backtrack_batch_tensors(cfg.B, du, dphi, dst)
    ctx.synchronize()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    dom = ctx.kernel_stats(0)
    walk = ctx.kernel_stats(1)
    print(json.dumps({"config": cfg_name, "steps": steps, "ms_per_step": round(1e3 * el / steps, 4),
                      "per_s": round(steps / el, 1), "dominant": [dom[2], round(dom[0] / max(1, dom[1]), 4)],
                      "walk": [walk[2], round(walk[0] / max(1, walk[1]), 4)], "status": int(dst.item()),
                      "diag": [int(d) for d in ctx.diagnostics()]}), flush=True)
