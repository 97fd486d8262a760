"""C5 batch timings of the fused separable DP variants (k_fsep2 with S row segments vs the one-lane-per-row
k_fsep_run): kernel time per launch (HIP events) at K restarts.  Usage: python scripts/bench_fsep.py [K ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

cfg = CONFIGS["C5"]
lt = cfg.levels()
Ks = [int(x) for x in sys.argv[1:]] or [1024, 128]
base = []
for k in range(max(Ks)):
    _, df, uo = make_inputs(cfg, k=k, levels=lt)
    base.append((df, uo))
for K in Ks:
    ddf = torch.tensor(np.ascontiguousarray(np.stack([base[k][0].T for k in range(K)])), dtype=torch.float64,
                       device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([base[k][1].T for k in range(K)])), dtype=torch.float64,
                       device="cuda")
    ref = None
    for seg in (-1, 1, 0, 2, 4, 8):
        ctx = native.Context(0)
        ctx.set_levels(lt)
        ctx.set_cost(cfg.p, cfg.beta)
        ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_FUSED_SEPARABLE)
        ctx.set_option(native.MIOC_OPT_FSEP_SEGMENTS, seg)
        ctx.set_option(native.MIOC_OPT_TIMING, 1)
        ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
        ctx.synchronize()
        ctx.reset_stats()
        for _ in range(3):
            ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
        ctx.synchronize()
        ms, n, name = ctx.kernel_stats(0)
        d = ctx.diagnostics()
        du = torch.empty_like(ddf)
        dphi = torch.empty(K, dtype=torch.float64, device="cuda")
        ctx.backtrack_batch_tensors(cfg.B, du, dphi, None)
        ctx.synchronize()
        out = (du.cpu().numpy(), dphi.cpu().numpy())
        same = "" if ref is None else ("  same" if all(np.array_equal(a, b) for a, b in zip(out, ref)) else "  DIFF")
        ref = ref or out
        print(f"K={K:5d} seg={seg:2d} {name:10s} {ms / n:9.3f} ms/launch = {K * n / ms * 1e3:9.1f} subproblems/s "
              f"({1e3 * ms / n / (cfg.nt - 1):.3f} us/step) segments={d[8]} occupancy={d[7]} redo={d[6]} "
              f"near-tie scans={d[0]} other scans={d[1]}{same}",
              flush=True)
        ctx.close()
