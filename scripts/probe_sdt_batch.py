"""Separable transform with K subproblems in one persistent launch: time per DP step and equality with single runs.
python probe_sdt_batch.py NT K REPS"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt, K, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cfg = CONFIGS["C4"]
lt = cfg.levels()
dfs, uos = [], []
for k in range(K):
    _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=lt)
    dfs.append(df)
    uos.append(uo)
ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
du = torch.empty_like(ddf)
dphi = torch.empty(K, dtype=torch.float64, device="cuda")
dst = torch.empty(K, dtype=torch.int32, device="cuda")
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
torch.cuda.synchronize()
t = []
for r in range(reps + 1):
    ctx.reset_stats()
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    ctx.synchronize()
    ms, n, name = ctx.kernel_stats(0)
    if r:
        t.append(1e3 * ms / (nt - 1))
ctx.backtrack_batch_tensors(cfg.B, du, dphi, dst)
ctx.synchronize()
print(f"K={K} nt={nt} {name}: us per DP step (all K) {' '.join(f'{x:.2f}' for x in t)} | per subproblem-step "
      f"{min(t) / K:.2f} us", flush=True)
ctx.close()
if K > 1:
    ub = du.cpu().numpy()
    for k in range(K):
        single = native.Context(0); single.set_levels(lt); single.set_cost(1, cfg.beta)
        single.bellman(dfs[k], uos[k], cfg.B, cfg.dt)
        u, ps, _ = single.backtrack(cfg.B)
        ok = np.array_equal(ub[k].T, u) and dphi[k].item() == ps and dst[k].item() == 0
        print(f"k={k}: batch == single: {ok} (phi {dphi[k].item()!r} vs {ps!r})", flush=True)
        assert ok
        single.close()
