"""ODE-constrained objectives (the gradient producers feeding the DP) and the reference's instances.

Mirrors the reference:
  AbstractODEObjective, eval_f_helper / eval_df_helper   julia_opt/ODEObjective.jl:62, :125-184
  LVMObj   (fishing, Lotka-Volterra)                     julia_opt/example_fishing.jl:14-92
  DTMObj   (double tank multimode)                       julia_opt/example_doubletank.jl:14-82
  VPOObj   (Van der Pol, binary variant)                 julia_opt/example_vanderpol.jl:14-81

These run on the host (numpy); they are the plumbing around the hot path (SURVEY §8 f rank 2),
not part of it.
"""
from __future__ import annotations

import numpy as np

from .iterators import bounded_sum_iterator
from .objective import AbstractObjectiveLazy


class AbstractODEObjective(AbstractObjectiveLazy):
    """min ∫ G(t, y, u) dt  s.t.  y' = F(t, y, u), y(T0) = y0 -- explicit Euler + trapezoid."""

    def __init__(self, T0, T1, nt, V, iterator, state0):
        self.T0, self.T1, self.nt = float(T0), float(T1), int(nt)
        self.V = [list(v) for v in V]
        self.iterator = iterator
        self.state0 = np.array(state0, dtype=np.float64)
        self.nu = 0
        self.nv = len(self.V)
        self.ny = len(self.state0)
        self.nx = self.nu + self.nv
        self.tau = (self.T1 - self.T0) / self.nt
        self._init_fields(self.nx, self.nt)
        self.state = np.zeros((self.ny, self.nt), order="F")
        self.adjoint = np.zeros((self.ny, self.nt), order="F")

    # user hooks (ODEObjective.jl:243-248)
    def F(self, Fval, i, y, x): raise NotImplementedError
    def Fy(self, Fyval, i, y, x): raise NotImplementedError
    def Fu(self, Fuval, i, y, x): raise NotImplementedError
    def G(self, i, y, x): raise NotImplementedError
    def Gy(self, Gyval, i, y, x): raise NotImplementedError
    def Gu(self, Guval, i, y, x): return None

    def i2t(self, i):
        return self.T0 + i * self.tau

    def eval_f_helper(self, x, cache):
        """ODEObjective.jl:125-150."""
        Fval = np.zeros(self.ny)
        state = self.state0.copy()
        fval = 0.5 * self.G(0, self.state0, x[:, 0])
        for i in range(self.nt):
            self.F(Fval, i, state, x[:, i])
            state += self.tau * Fval
            if cache:
                self.state[:, i] = state
            if i < self.nt - 1:
                fval += self.G(i + 1, state, x[:, i + 1])
            else:
                fval += 0.5 * self.G(self.nt - 1, state, x[:, self.nt - 1])
        fval *= self.tau
        return fval

    def eval_df_helper(self):
        """ODEObjective.jl:153-184 (explicit Euler for the adjoint, then df = Gu - Fu' λ)."""
        ny, nx, nt, tau = self.ny, self.nx, self.nt, self.tau
        Fyval = np.zeros((ny, ny))
        Gyval = np.zeros(ny)
        Fuval = np.zeros((ny, nx))
        Guval = np.zeros(nx)
        self.Gy(Gyval, nt, self.state[:, nt - 1], self.x[:, nt - 1])
        self.adjoint[:, nt - 1] = -0.5 * tau * Gyval
        for i in range(nt - 1, 0, -1):  # Julia i = nt-1:-1:1 (1-based)
            self.Gy(Gyval, i, self.state[:, i - 1], self.x[:, i])
            self.Fy(Fyval, i, self.state[:, i - 1], self.x[:, i])
            self.adjoint[:, i - 1] = self.adjoint[:, i] + tau * (Fyval.T @ self.adjoint[:, i] - Gyval)
        self.df[:, :] = 0.0
        for i in range(1, nt + 1):
            state = self.state0 if i == 1 else self.state[:, i - 2]
            self.Fu(Fuval, i - 1, state, self.x[:, i - 1])
            self.Gu(Guval, i - 1, state, self.x[:, i - 1])
            self.df[:, i - 1] -= Fuval.T @ self.adjoint[:, i - 1]
            self.df[:, i - 1] += Guval


class LVMObj(AbstractODEObjective):
    """Lotka-Volterra fishing problem (julia_opt/example_fishing.jl:14-92)."""

    def __init__(self, nt=1200, T0=0.0, T1=12.0):
        V = [[0, 1], [0, 1], [0, 1]]
        super().__init__(T0, T1, nt, V, bounded_sum_iterator(V, 1, 1), [0.5, 0.7])
        self.alpha = self.beta = self.gamma = self.delta = self.c1 = self.c2 = 1.0
        self.v1 = np.array([0.2, 0.4, 0.01])
        self.v2 = np.array([0.1, 0.2, 0.1])

    def F(self, Fval, i, y, x):
        Fval[0] = y[0] * (self.alpha - self.beta * y[1] - self.c1 * np.sum(x * self.v1))
        Fval[1] = y[1] * (-self.gamma + self.delta * y[0] - self.c2 * np.sum(x * self.v2))

    def Fy(self, Fyval, i, y, x):
        Fyval[0, 0] = self.alpha - self.beta * y[1] - self.c1 * np.sum(x * self.v1)
        Fyval[0, 1] = y[0] * -self.beta
        Fyval[1, 0] = y[1] * self.delta
        Fyval[1, 1] = -self.gamma + self.delta * y[0] - self.c2 * np.sum(x * self.v2)

    def Fu(self, Fuval, i, y, x):
        Fuval[0, :] = y[0] * -self.c1 * self.v1
        Fuval[1, :] = y[1] * -self.c2 * self.v2

    def G(self, i, y, x):
        return 0.5 * (y[0] - 1.0) ** 2 + 0.5 * (y[1] - 1.0) ** 2

    def Gy(self, Gyval, i, y, x):
        Gyval[0] = y[0] - 1.0
        Gyval[1] = y[1] - 1.0


class DTMObj(AbstractODEObjective):
    """Double tank multimode problem (julia_opt/example_doubletank.jl:14-82)."""

    def __init__(self, nt=1000, T0=0.0, T1=10.0):
        V = [[0, 1], [0, 1], [0, 1]]
        super().__init__(T0, T1, nt, V, bounded_sum_iterator(V, 1, 1), [2.0, 2.0])
        self.k1, self.k2 = 2.0, 3.0
        self.c = np.array([1.0, 0.5, 2.0])

    def F(self, Fval, i, y, x):
        Fval[0] = self.c @ x - np.sqrt(y[0])
        Fval[1] = np.sqrt(y[0]) - np.sqrt(y[1])

    def Fy(self, Fyval, i, y, x):
        Fyval[0, 0] = -1 / (2 * np.sqrt(y[0]))
        Fyval[0, 1] = 0.0
        Fyval[1, 0] = 1 / (2 * np.sqrt(y[0]))
        Fyval[1, 1] = -1 / (2 * np.sqrt(y[1]))

    def Fu(self, Fuval, i, y, x):
        Fuval[0, :] = self.c
        Fuval[1, :] = 0.0

    def G(self, i, y, x):
        return self.k1 * (y[1] - self.k2) ** 2

    def Gy(self, Gyval, i, y, x):
        Gyval[0] = 0.0
        Gyval[1] = 2 * self.k1 * (y[1] - self.k2)


class VPOObj(AbstractODEObjective):
    """Van der Pol oscillator, binary variant (julia_opt/example_vanderpol.jl:14-81)."""

    def __init__(self, nt=2000, T0=0.0, T1=20.0):
        V = [[0, 1], [0, 1], [0, 1]]
        super().__init__(T0, T1, nt, V, bounded_sum_iterator(V, 1, 1), [1.0, 0.0])
        self.c = np.array([-1.0, 0.75, -2.0])

    def F(self, Fval, i, y, x):
        Fval[0] = y[1]
        Fval[1] = (1 - y[0] ** 2) * y[1] * (self.c @ x) - y[0]

    def Fy(self, Fyval, i, y, x):
        s = self.c @ x
        Fyval[0, 0] = 0.0
        Fyval[0, 1] = 1.0
        Fyval[1, 0] = -2 * y[0] * y[1] * s - 1
        Fyval[1, 1] = (1 - y[0] ** 2) * s

    def Fu(self, Fuval, i, y, x):
        Fuval[0, :] = 0.0
        Fuval[1, :] = self.c * (1 - y[0] ** 2) * y[1]

    def G(self, i, y, x):
        return y[0] ** 2 + y[1] ** 2

    def Gy(self, Gyval, i, y, x):
        Gyval[0] = 2 * y[0]
        Gyval[1] = 2 * y[1]
