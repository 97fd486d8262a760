"""Debug: the last steps of the nt=64 C4 fixture (the steps next to the terminal) as their own problem, oracle vs
device cell by cell (persistent separable, per-step separable, pyramid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS
from oracle.oracle import OracleC, Levels, P_ONE
z = np.load(os.path.join(ROOT, "tests", "golden", "hashed", "c4_4096lv_p1_nt64_uhash.npz"))
t0 = int(sys.argv[1]) if len(sys.argv) > 1 else 51
cfg = CONFIGS["C4"]; lt = cfg.levels()
df, uo = z["df"][:, t0:], z["u_old"][:, t0:]
n = df.shape[1]
lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
phi, U = OracleC().bellman(lv, df, uo, cfg.B, P_ONE, cfg.beta, cfg.dt)
print("oracle done, nt", n, flush=True)
for name, algo, persist in (("persistent", 4, 1), ("steps", 4, 0), ("pyramid", 3, 1)):
    ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
    ctx.set_option(native.MIOC_OPT_ALGO, algo); ctx.set_option(native.MIOC_OPT_PERSIST, persist)
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    for i in range(n - 1):
        d, o = ctx.argmin_table(i), U[:, :, i]
        w = o >= 0
        mis = w & (d != o)
        extra = (~w) & (d >= 0)
        if mis.any() or extra.any():
            cs, gs = np.nonzero(mis)
            ce, ge = np.nonzero(extra)
            print(f"{name} step {i}: {mis.sum()} mismatched written cells (c,g,dev,ref) "
                  f"{[(int(c), int(g), int(d[c, g]), int(o[c, g])) for c, g in zip(cs[:4], gs[:4])]}; "
                  f"{extra.sum()} extra device cells {[(int(c), int(g), int(d[c, g])) for c, g in zip(ce[:4], ge[:4])]}")
    print(name, "diag", ctx.diagnostics(), flush=True)
    ctx.close()
