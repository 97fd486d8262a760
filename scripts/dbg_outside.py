"""Debug: the 8x8x8 'outside' case (off-grid u_old) on the persistent separable kernel vs the per-step one vs the
oracle, per step, several runs and buffer counts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from mioc import native  # noqa: E402
from mioc.iterators import LevelTable  # noqa: E402
from oracle.oracle import P_ONE, Levels, OracleC  # noqa: E402

rng = np.random.default_rng(6)
lv = Levels.product([list(range(8))] * 3)
lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
n, B = 12, 20
df = rng.integers(-64, 65, size=(3, n)) / 64.0
uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(n)], dtype=np.float64).T
df = rng.standard_normal((3, n))
for i in rng.choice(n, size=5, replace=False):
    uo[:, i] = [-1.0, 8.0, 3.0]
beta, dt = 1e-3, 2.0 ** -10
oc = OracleC()
phi, U = oc.bellman(lv, df, uo, B, P_ONE, beta, dt)
for persist, nb, rep in [(0, 64, 0), (1, 64, 0), (1, 64, 1), (1, 4, 0), (1, 64, 2)]:
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(None, beta, p_kind=P_ONE)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_SEPARABLE)
    ctx.set_option(native.MIOC_OPT_PERSIST, persist)
    ctx.set_option(native.MIOC_OPT_SDT_BUFFERS, nb)
    ctx.bellman(df, uo, B, dt)
    ctx.synchronize()
    bad = []
    for i in range(n - 1):
        d = ctx.argmin_table(i)
        o = U[:, :, i]
        m = o >= 0
        nb_ = int(np.sum(m & (d != o)))
        bad.append(nb_)
        if nb_ and persist:
            w = np.argwhere(m & (d != o))
            print(f"   step {i}: rows {sorted(set(w[:, 0].tolist()))[:12]} ranks {w[:6, 1].tolist()}")
    print(f"persist={persist} NB={nb} rep={rep}: mismatches per step {bad} diag {ctx.diagnostics()} algo {ctx.last_algo()}",
          flush=True)
    ctx.close()
