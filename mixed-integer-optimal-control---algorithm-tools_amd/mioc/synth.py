"""Seeded synthetic subproblem inputs for the benchmark configurations (SURVEY.md §8 d).

Every config restates the reference's level sets and ``main()`` presets (multi-trust.jl:181-195):
  C1 fishing     M=3, 3-of-8 SOS1 levels (example_fishing.jl:22-24), nt=512,  Δt=12/512,  Δ⁰=2, β=1e-4, p=Inf
  C2 doubletank  M=3, SOS1 (example_doubletank.jl:20-22),            nt=4096, Δt=10/4096, Δ⁰=2, β=1e-5, p=Inf
  C3 vanderpol   M=3, SOS1 (example_vanderpol.jl:20-22),             nt=16384,Δt=20/16384,Δ⁰=1, β=0.1,  p=Inf
  C4 synthetic   M=4, levels 0..7 each, product (4096 tuples),       nt=65536,Δt=2^-16,   Δ⁰=2^-8 (B=256),
                 β=1e-3, p=1 (p=Inf variant)
  C5 batch       heat-shaped [0..5]^2 product (example_heat.jl:42-44), nt=4096, Δt=2^-12, B=256, p=1, β=1e-3
df ~ N(0,1) (x0.1 for C1-C3), u_old piecewise constant with floor(nt/10) jumps over admissible
tuples (the shape of rand_func_int, HelpFunctions.jl:204-225).  numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .iterators import LevelTable, bounded_sum_iterator, product_iterator


@dataclass
class SubproblemConfig:
    name: str
    nu: list
    iterator_kind: str  # "product" or "sos1"
    nt: int
    dt: float
    Delta0: float
    beta: float
    p: float
    df_scale: float = 1.0
    seed_df: int = 0xC4DF
    seed_u: int = 0xC4A0

    @property
    def B(self):
        return int(math.floor(self.Delta0 / self.dt))

    def levels(self):
        it = product_iterator(self.nu) if self.iterator_kind == "product" else bounded_sum_iterator(self.nu, 1, 1)
        return LevelTable(self.nu, it)


SOS1 = [[0, 1], [0, 1], [0, 1]]

CONFIGS = {
    "C1": SubproblemConfig("fishing", SOS1, "sos1", 512, 12 / 512, 2.0, 1e-4, math.inf, 0.1, 0xC1DF, 0xC1A0),
    "C2": SubproblemConfig("doubletank", SOS1, "sos1", 4096, 10 / 4096, 2.0, 1e-5, math.inf, 0.1, 0xC2DF, 0xC2A0),
    "C3": SubproblemConfig("vanderpol", SOS1, "sos1", 16384, 20 / 16384, 1.0, 0.1, math.inf, 0.1, 0xC3DF, 0xC3A0),
    "C4": SubproblemConfig("synthetic", [list(range(8))] * 4, "product", 65536, 2.0 ** -16, 2.0 ** -8, 1e-3, 1,
                           1.0, 0xC4DF, 0xC4A0),
    "C5": SubproblemConfig("batch-heat", [list(range(6))] * 2, "product", 4096, 2.0 ** -12, 2.0 ** -4, 1e-3, 1,
                           1.0, 0xC5000, 0xC5800),
}


def synthetic_df(M, nt, seed, scale=1.0):
    g = np.random.Generator(np.random.PCG64(seed))
    return np.asfortranarray(g.standard_normal((M, nt)) * scale)


def synthetic_u_old(levels: LevelTable, nt, seed, jumps=None):
    g = np.random.Generator(np.random.PCG64(seed))
    jumps = nt // 10 if jumps is None else jumps
    jumps = min(jumps, max(nt - 1, 0))
    t = np.sort(g.choice(np.arange(1, nt), size=jumps, replace=False)) if jumps else np.array([], dtype=np.int64)
    seg = g.integers(levels.L, size=jumps + 1)
    idx = np.searchsorted(t, np.arange(nt), side="right")
    return np.asfortranarray(levels.nuval[seg[idx]].T.copy())


def make_inputs(cfg: SubproblemConfig, k=0, nt=None, levels=None):
    """(levels, df, u_old) for restart k of a config; nt may be truncated for parity tests."""
    levels = cfg.levels() if levels is None else levels
    nt = cfg.nt if nt is None else nt
    df = synthetic_df(levels.M, nt, cfg.seed_df + k, cfg.df_scale)
    u = synthetic_u_old(levels, nt, cfg.seed_u + k)
    return levels, df, u
