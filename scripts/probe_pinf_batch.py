"""p=Inf collapse on K restarts (C2 / C3 shapes): per-kernel times of bellman (prep + recursion) and backtrack
(start + walk), whole-batch wall time, subproblems/s, and a digest of u / Φ* (equal across library builds; MIOC_LIB
selects one).  python probe_pinf_batch.py CFG K [K ...]"""
import hashlib, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
import numpy as np
import torch
from mioc import native
from mioc.synth import CONFIGS, make_inputs
cfg = CONFIGS[sys.argv[1]]
lt = cfg.levels()
for K in [int(x) for x in sys.argv[2:]]:
    g = torch.Generator(device="cuda").manual_seed(K)
    ddf = torch.randn(K, cfg.nt, lt.M, dtype=torch.float64, device="cuda", generator=g) * cfg.df_scale
    uos = [make_inputs(cfg, k=k, nt=cfg.nt, levels=lt)[2] for k in range(min(K, 64))]
    duo = torch.tensor(np.ascontiguousarray(np.stack([uos[k % len(uos)].T for k in range(K)])),
                       dtype=torch.float64, device="cuda")
    du = torch.empty_like(ddf)
    dphi = torch.empty(K, dtype=torch.float64, device="cuda")
    ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(cfg.p, cfg.beta)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    walls = []
    for r in range(3):
        ctx.reset_stats()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
        ctx.backtrack_batch_tensors(cfg.B, du, dphi)
        ctx.synchronize()
        walls.append(time.perf_counter() - t0)
    st = [ctx.kernel_stats(w) for w in (0, 2, 1)]
    dg = hashlib.sha256(du.cpu().numpy().tobytes() + dphi.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{os.path.basename(os.environ.get('MIOC_LIB', 'libmioc.so'))} {sys.argv[1]} K={K} digest {dg}: wall {min(walls) * 1e3:.2f} ms -> {K / min(walls):.1f} subproblems/s | " +
          " | ".join(f"{n} {ms:.2f} ms/{c}" for ms, c, n in st), flush=True)
    ctx.close()
