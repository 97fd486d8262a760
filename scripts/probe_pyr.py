"""Probe the p=1 pyramid on the C4 config: diagnostics counters and per-step kernel time (HIP events)."""
import os, sys, time, math
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 512
algo = int(sys.argv[2]) if len(sys.argv) > 2 else native.MIOC_ALGO_PYRAMID
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta); ctx.set_option(native.MIOC_OPT_ALGO, algo)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
for rep in range(2):
    ctx.reset_stats()
    t0 = time.perf_counter(); ctx.bellman(df, uo, cfg.B, cfg.dt); t1 = time.perf_counter()
    ms, n, name = ctx.kernel_stats(0)
    print(f"rep {rep}: {name} {n} launches, {1e3*ms/max(n,1):.2f} us/step (events), wall {1e3*(t1-t0):.1f} ms, diag {ctx.diagnostics()}")
u, phi, _ = ctx.backtrack(cfg.B)
print("phi*", phi)
