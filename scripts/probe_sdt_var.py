"""Run-to-run spread of k_sdt_run at full C4 (nt = 65536): each call of this script is one process (one context, its own
allocations); it times REPS bellman calls and prints each, so that within-process and across-process spread can be
told apart.  Usage: python scripts/probe_sdt_var.py [reps] [nt]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))
sys.path.insert(0, ROOT)
from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
cfg = CONFIGS["C4"]
lt = cfg.levels()
_, df, uo = make_inputs(cfg, nt=nt, levels=lt)
with native.Context(0) as ctx:
    ctx.set_levels(lt)
    ctx.set_cost(1, cfg.beta)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    out = []
    for _ in range(reps):
        ctx.reset_stats()
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        ctx.synchronize()
        ms, n, name = ctx.kernel_stats(0)
        out.append(round(1e3 * ms / (nt - 1), 3))
    print(json.dumps({"pid": os.getpid(), "us_per_step": out}), flush=True)
