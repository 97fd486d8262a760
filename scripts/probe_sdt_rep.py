"""Repeated k_sdt_run timings (persistent separable transform) in one process: python probe_sdt_rep.py NT REPS.
MIOC_LIB selects the library build (A/B comparisons of two builds in one GPU call)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt, reps = int(sys.argv[1]), int(sys.argv[2])
cfg = CONFIGS["C4"]
lt = cfg.levels()
_, df, uo = make_inputs(cfg, nt=nt, levels=lt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
out = []
for r in range(reps + 1):
    ctx.reset_stats()
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    ctx.synchronize()
    ms, n, name = ctx.kernel_stats(0)
    if r:
        out.append(1e3 * ms / (nt - 1))
print(os.path.basename(os.environ.get("MIOC_LIB", "libmioc.so")), name, "us/step:", " ".join(f"{x:.2f}" for x in out),
      f"| min {min(out):.2f} median {sorted(out)[len(out) // 2]:.2f}", flush=True)
ctx.close()
