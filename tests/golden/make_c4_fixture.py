"""Generate tests/golden/hashed/c4_4096lv_p1_nt64_uhash.npz: the BASELINE roofline shape (C4: 8^4 = 4096 levels,
B = 256, p = 1, seeded inputs of mioc.synth) truncated to nt = 64, solved by the C oracle (the restatement of
HelpFunctions.jl:20-124).  63 recursion steps: every rotation of k_sdt_run's four staging buffers, and row B's
two-step lag, many times over.  Stored: the inputs, sha256 of every step's argmin table U in the reference
layout (int32 [B+1, 4096], -1 where the reference writes nothing), and u / Φ* for B' in {256, 128, 7}.
Run:  python tests/golden/make_c4_fixture.py   (about 2 minutes on one core)
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))

from oracle.oracle import P_ONE, Levels, OracleC  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

NT = 64
BPS = (256, 128, 7)


def table_hash(t):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(t, dtype=np.int32).tobytes()).digest(), dtype=np.uint8)


def main():
    cfg = CONFIGS["C4"]
    lt, df, uo = make_inputs(cfg, nt=NT)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    t0 = time.time()
    phi, U = OracleC().bellman(lv, df, uo, cfg.B, P_ONE, cfg.beta, cfg.dt)
    print(f"oracle DP: {time.time() - t0:.1f} s")
    hashes = np.stack([table_hash(U[:, :, i]) for i in range(NT - 1)])
    us, ps = [], []
    for Bp in BPS:
        u, p = OracleC().backtrack(lv, uo, phi, U, cfg.B, Bp)
        us.append(u)
        ps.append(p)
    np.savez(os.path.join(HERE, "hashed", "c4_4096lv_p1_nt64_uhash.npz"), df=df, u_old=uo, B=np.array([cfg.B]),
             beta=np.array([cfg.beta]), dt=np.array([cfg.dt]), budgets=np.array(BPS), u=np.stack(us),
             phi_star=np.array(ps), u_hash=hashes, written=np.array([int((U >= 0).sum())]))
    print("phi*", ps, "written cells", int((U >= 0).sum()))


if __name__ == "__main__":
    main()
