"""k_sdt_run vs k_sdt_step total time at several nt (normal build), second call of each."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
cfg = CONFIGS["C4"]
lt = cfg.levels()
for nt in [int(x) for x in sys.argv[1:]]:
    _, df, uo = make_inputs(cfg, nt=nt, levels=lt)
    for persist in (1, 0):
        ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
        ctx.set_option(native.MIOC_OPT_TIMING, 1); ctx.set_option(native.MIOC_OPT_PERSIST, persist)
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        ctx.synchronize(); ctx.reset_stats()
        t0 = time.perf_counter()
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        ctx.synchronize()
        wall = time.perf_counter() - t0
        ms, n, name = ctx.kernel_stats(0)
        u, phi, _ = ctx.backtrack(cfg.B)
        print(f"nt={nt} {name}: events {ms:.3f} ms ({1e3 * ms / (nt - 1):.2f} us/step), wall {1e3 * wall:.3f} ms, phi={phi!r} diag={ctx.diagnostics()}", flush=True)
        ctx.close()
