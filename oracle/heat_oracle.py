"""TEST INFRASTRUCTURE -- CPU oracle for the PDE heat objective's value and gradient.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, and only as the checker
(or the timed CPU baseline); the product path is mioc_heat_eval_device (mixed-integer-optimal-control---algorithm-
tools_amd/csrc/mioc_heat.hip).

A line-by-line restatement of julia_opt/PDEObjective.jl with the hooks of julia_opt/example_heat.jl, with the
reference's own operations: LU factors of StateMat = I + τ·M⁻¹A and of its transpose (example_heat.jl:113-115,
scipy.linalg.lu_factor = LAPACK getrf, the factorisation Julia's `lu` calls), one triangular solve pair per step.
Parity: the reference is Julia and cannot run here, and its repository holds no heat outputs, so this restatement is
pinned by the reference's own check of the gradient -- the finite-difference test of example_heat.jl:186-223
(tests/test_heat.py) -- and by the closed-form cost of the stationary state; parity with Julia's own floats is
unpinned.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla


class HeatOracle:
    def __init__(self, M_invA, M_invF, M, state0, yd, T0, T1, gamma):
        self.M_invA, self.M_invF, self.M = M_invA, M_invF, M
        self.state0, self.yd, self.gamma = state0, yd, gamma
        self.nt = yd.shape[1] - 1
        self.tau = (T1 - T0) / self.nt                                  # example_heat.jl:90
        N = M.shape[0]
        S = np.eye(N) + self.tau * M_invA                               # example_heat.jl:113
        self.SLU = sla.lu_factor(S)                                     # SMatLU = lu(StateMat)
        self.ALU = sla.lu_factor(S.T)                                   # AMatLU = lu(StateMat')

    def G(self, state, i):                                              # example_heat.jl:135-140
        v = state[:, i] - self.yd[:, i]
        return 0.5 * (v @ self.M) @ v

    def eval(self, x):
        """x: (nx, nt) (Julia's layout).  Returns (fval, df (nx, nt), state (N, nt+1))."""
        nt, tau = self.nt, self.tau
        xe = np.hstack([x, x[:, -1:]])                                  # PDEObjective.jl:145
        state = np.empty((self.M.shape[0], nt + 1))
        state[:, 0] = self.state0                                       # :130
        for i in range(1, nt + 1):                                      # :134-137
            state[:, i] = sla.lu_solve(self.SLU, state[:, i - 1] + tau * (self.M_invF @ xe[:, i - 1]))
        Gt = lambda i: self.gamma * np.sum(xe[:, i])                    # noqa: E731  example_heat.jl:143-145
        fval = 0.5 * (self.G(state, 0) + Gt(0))                         # PDEObjective.jl:148
        for i in range(1, nt):                                          # :149-151
            fval += self.G(state, i) + Gt(i)
        fval += 0.5 * (self.G(state, nt) + Gt(nt))                      # :152
        fval *= tau                                                     # :153
        adj = np.zeros_like(state)                                      # :163
        for i in range(nt - 1, -1, -1):                                 # :167-170
            Gy = self.M @ (state[:, i] - self.yd[:, i])                 # Gy! (example_heat.jl:152-155)
            adj[:, i] = sla.lu_solve(self.ALU, adj[:, i + 1] + tau * Gy)
        df = np.zeros(x.shape)                                          # :182
        for i in range(nt):                                             # :185-187
            df[:, i] += self.M_invF.T @ adj[:, i]
        for i in range(1, nt):                                          # :193-197 (Gu at i = 1 is not added)
            df[:, i] += self.gamma
        return fval, df, state


def eval_batch(args):
    """Worker of the CPU baseline (bench.py): (matrices, T0, T1, gamma, controls) -> [(fval, df)]; one process per
    worker, because concurrent LAPACK calls from threads of one process crash this image's BLAS."""
    mats, T0, T1, gamma, xs = args
    o = HeatOracle(*mats, T0, T1, gamma)
    return [o.eval(x)[:2] for x in xs]
