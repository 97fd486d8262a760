"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference (Julia) cannot run in this image and holds no fixtures for this path, so the fixtures
come from the oracle chain: exhaustive enumeration (exact arithmetic, dyadic inputs) for the KAT
cases, and the C oracle (cross-checked against the pure-Python twin where small enough) for the
config-shaped cases.  Run:  python tests/golden/make_golden.py
Each .npz holds only arrays (np.load(..., allow_pickle=False)):
  nu_counts, nu_values, tuples (L x M, 1-based), df, u_old, scalars [B, Bp, beta, dt, p_kind, p_int],
  wtab (weight table or empty), u (expected control), phi_star, source (0 enumeration, 1 C oracle)
"""
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"))

from oracle.oracle import (P_INF, P_INTLUT, P_ONE, Levels, OracleC, backtrack_py, bellman_py,  # noqa: E402
                           enumerate_kat)
from mioc.synth import CONFIGS, make_inputs  # noqa: E402


def save(name, lv, df, uo, B, Bp, beta, dt, pk, pint, wtab, u, phi, source):
    np.savez(os.path.join(HERE, name + ".npz"), nu_counts=lv.counts, nu_values=lv.values, tuples=lv.tuples,
             df=np.asarray(df, dtype=np.float64), u_old=np.asarray(uo, dtype=np.float64),
             scalars=np.array([B, Bp, beta, dt, pk, pint], dtype=np.float64),
             wtab=np.zeros(0) if wtab is None else np.asarray(wtab, dtype=np.float64),
             u=np.asarray(u, dtype=np.float64), phi_star=np.array([phi]), source=np.array([source]))
    print(f"  {name}: M={lv.M} L={lv.L} nt={df.shape[1]} B={B} Bp={Bp} p_kind={pk} phi*={phi!r}")


def kat_cases():
    rng = np.random.default_rng(20250614)
    specs = [
        ("kat_sos1_pinf", [[0, 1], [0, 1], [0, 1]], "sos1", P_INF, 5, 3),
        ("kat_sos1_p1", [[0, 1], [0, 1], [0, 1]], "sos1", P_ONE, 5, 4),
        ("kat_prod2x3_p1", [[0, 1, 2], [0, 1]], "prod", P_ONE, 4, 4),
        ("kat_prod2x3_pinf", [[0, 1, 2], [0, 1]], "prod", P_INF, 4, 3),
        ("kat_gap_levels_p1", [[-2, 0, 3]], "prod", P_ONE, 6, 7),
        ("kat_prod3_p2", [[0, 1, 2]], "prod", P_INTLUT, 6, 5),
        ("kat_ties_zero_df", [[0, 1], [0, 1]], "prod", P_ONE, 5, 3),
    ]
    for name, nu, kind, pk, n, B in specs:
        lv = Levels.product(nu) if kind == "prod" else Levels.bounded_sum(nu, 1, 1)
        if name == "kat_ties_zero_df":
            df = np.zeros((lv.M, n))
        else:
            df = rng.integers(-8, 9, size=(lv.M, n)) / 8.0
        uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(n)], dtype=np.float64).T
        beta, dt = 0.25, 0.5
        pint, wtab = 1, None
        if pk == P_INTLUT:
            pint = 2
            wtab = np.array([0.0, 1.0, 1.5, 1.75, 2.0, 2.25, 2.5, 2.75, 3.0])  # dyadic stand-in weights
        Bp = max(0, B - 1)
        u, v = enumerate_kat(lv, df, uo, B, Bp, pk, beta, dt, p_int=pint, wtab=wtab)
        phi, U = bellman_py(lv, df, uo, B, pk, beta, dt, p_int=pint, wtab=wtab)
        u2, p2 = backtrack_py(lv, uo, phi, U, B, Bp)
        assert np.array_equal(u, u2) and float(v) == p2, name
        save(name, lv, df, uo, B, Bp, beta, dt, pk, pint, wtab, u, float(v), 0)


def config_cases(oc):
    specs = [
        ("c1_fishing_nt96", "C1", 96, None, None),
        ("c2_doubletank_nt256", "C2", 256, 60, None),
        ("c3_vanderpol_nt128", "C3", 128, 40, None),
        ("c5_heat36_p1_nt48", "C5", 48, 24, None),
        ("c5_heat36_p2lut_nt32", "C5", 32, 16, 2),
        ("c4_4096lv_p1_nt5", "C4", 5, None, None),
        ("c4_4096lv_pinf_nt9", "C4", 9, None, math.inf),
    ]
    for name, key, nt, Bcap, pover in specs:
        cfg = CONFIGS[key]
        lvt, df, uo = make_inputs(cfg, nt=nt)
        lv = Levels(lvt.nu, [tuple(t) for t in lvt.tuples])
        p = cfg.p if pover is None else pover
        B = cfg.B if Bcap is None else min(cfg.B, Bcap)
        pint, wtab = 1, None
        if p == math.inf:
            pk = P_INF
        elif p == 1:
            pk = P_ONE
        else:
            pk, pint = P_INTLUT, int(p)
            maxkey = sum((max(v) - min(v)) ** pint for v in lv.nu)
            wtab = np.array([float(s) ** (1.0 / pint) for s in range(maxkey + 1)])
        t0 = time.time()
        phi, U = oc.bellman(lv, df, uo, B, pk, cfg.beta, cfg.dt, p_int=pint, wtab=wtab)
        Bp = B if name.endswith("nt5") or name.endswith("nt9") else max(0, B // 2)
        u, ps = oc.backtrack(lv, uo, phi, U, B, Bp)
        if lv.L * lv.L * nt * (B + 1) < 3e6:
            phi2, U2 = bellman_py(lv, df, uo, B, pk, cfg.beta, cfg.dt, p_int=pint, wtab=wtab)
            assert np.array_equal(phi, phi2) and np.array_equal(U, U2), name
        save(name, lv, df, uo, B, Bp, cfg.beta, cfg.dt, pk, pint, wtab, u, ps, 1)
        print(f"    ({time.time() - t0:.1f} s)")


if __name__ == "__main__":
    print("enumeration KATs:")
    kat_cases()
    print("config-shaped (C oracle):")
    config_cases(OracleC())
