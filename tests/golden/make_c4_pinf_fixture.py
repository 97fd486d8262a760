"""Generate tests/golden/hashed/c4_4096lv_pinf_nt200.npz: the BASELINE roofline shape (C4: 8^4 = 4096 levels, B = 256,
seeded inputs of mioc.synth) at p = Inf, truncated to nt = 200, solved by the C oracle (the restatement of
HelpFunctions.jl:20-124; at p = Inf every transition costs beta, HelpFunctions.jl:63-67).  199 recursion steps: more
than three of k_pinf_recur_mc's 64-step hand-off chunks and a wrap of its 128-slot LDS ring.  Stored: the inputs, and
u / Φ* for B' in BPS (the backtrack walks every step's argmin along its path).
Run:  python tests/golden/make_c4_pinf_fixture.py   (a few minutes on 8 cores: OpenMP over the target levels of each
step, bit-identical to the single-threaded oracle)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))

from oracle.oracle import P_INF, Levels, OracleC  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

NT = 200
BPS = (256, 128, 64, 7, 0)


def main():
    cfg = CONFIGS["C4"]
    lt, df, uo = make_inputs(cfg, nt=NT)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    oc = OracleC()
    t0 = time.time()
    phi, U = oc.bellman(lv, df, uo, cfg.B, P_INF, cfg.beta, cfg.dt, threads=os.cpu_count() or 1)
    print(f"oracle DP: {time.time() - t0:.1f} s")
    us, ps = [], []
    for Bp in BPS:
        u, p = oc.backtrack(lv, uo, phi, U, cfg.B, Bp)
        us.append(u)
        ps.append(p)
    np.savez(os.path.join(HERE, "hashed", "c4_4096lv_pinf_nt200.npz"), df=df, u_old=uo, B=np.array([cfg.B]),
             beta=np.array([cfg.beta]), dt=np.array([cfg.dt]), budgets=np.array(BPS), u=np.stack(us),
             phi_star=np.array(ps), switches=np.array([int((np.abs(np.diff(u, axis=1)).sum(axis=0) > 0).sum())
                                                       for u in us]))
    print("phi*", ps)


if __name__ == "__main__":
    main()
