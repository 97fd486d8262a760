"""CPU oracle (test infrastructure only) for the ODE gradient producer of SURVEY §8 f2.

A scalar restatement -- plain Python floats, one operation at a time, no numpy, no BLAS -- of

  eval_f_helper    julia_opt/ODEObjective.jl:125-150   explicit Euler state + trapezoid objective
  eval_df_helper   julia_opt/ODEObjective.jl:153-184   explicit Euler adjoint, df = Gu - Fu' * adjoint

with the user hooks of the three ODE examples the reference's main() runs (multi-trust.jl:181-189):

  fishing      julia_opt/example_fishing.jl:56-92     (LVMObj, Lotka-Volterra, state0 = [0.5, 0.7], T = 12)
  doubletank   julia_opt/example_doubletank.jl:48-82  (DTMObj, state0 = [2, 2], T = 10)
  vanderpol    julia_opt/example_vanderpol.jl:48-81   (VPOObj, state0 = [1, 0], T = 20)

It shares no code with the product's host mirror (mioc/ode.py) and is imported only by tests/, as the checker of
the device producer (mioc_ode_eval_device).  Julia evaluates `sum(x .* v)` left to right for three terms; `c' * x`
and `Fyval' * adjoint` go through BLAS in Julia, whose rounding (FMA use) is not pinned here, so the device is held to
a relative tolerance on df and J, not bit equality.  The oracle itself is pinned the way the reference pins its own
gradients (`test_df`, example_fishing.jl:94-123 and the doubletank / vanderpol twins): the directional derivative
tau * sum_i df[:, i]' h[:, i] must match finite differences of eval_f (`fd_check`).
"""
from __future__ import annotations

import math

# example constants, as in the reference structs (example_*.jl:14-46)
FISHING = dict(T0=0.0, T1=12.0, state0=(0.5, 0.7), alpha=1.0, beta=1.0, gamma=1.0, delta=1.0, c1=1.0, c2=1.0,
               v1=(0.2, 0.4, 0.01), v2=(0.1, 0.2, 0.1))
DOUBLETANK = dict(T0=0.0, T1=10.0, state0=(2.0, 2.0), k1=2.0, k2=3.0, c=(1.0, 0.5, 2.0))
VANDERPOL = dict(T0=0.0, T1=20.0, state0=(1.0, 0.0), c=(-1.0, 0.75, -2.0))


def _sum3(a, b):
    """Julia's sum(a .* b) for three entries: ((a1 b1 + a2 b2) + a3 b3)."""
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


class _Fishing:
    """example_fishing.jl:56-92."""
    P = FISHING

    def F(self, y, x):
        p = self.P
        return (y[0] * (p["alpha"] - p["beta"] * y[1] - p["c1"] * _sum3(x, p["v1"])),
                y[1] * (-p["gamma"] + p["delta"] * y[0] - p["c2"] * _sum3(x, p["v2"])))

    def Fy(self, y, x):
        p = self.P
        return ((p["alpha"] - p["beta"] * y[1] - p["c1"] * _sum3(x, p["v1"]), y[0] * -p["beta"]),
                (y[1] * p["delta"], -p["gamma"] + p["delta"] * y[0] - p["c2"] * _sum3(x, p["v2"])))

    def Fu(self, y, x):
        p = self.P
        return (tuple(y[0] * -p["c1"] * v for v in p["v1"]), tuple(y[1] * -p["c2"] * v for v in p["v2"]))

    def G(self, y, x):
        return 0.5 * (y[0] - 1.0) ** 2 + 0.5 * (y[1] - 1.0) ** 2

    def Gy(self, y, x):
        return (y[0] - 1.0, y[1] - 1.0)


class _DoubleTank:
    """example_doubletank.jl:48-82."""
    P = DOUBLETANK

    def F(self, y, x):
        c = self.P["c"]
        return (_sum3(c, x) - math.sqrt(y[0]), math.sqrt(y[0]) - math.sqrt(y[1]))

    def Fy(self, y, x):
        return ((-1 / (2 * math.sqrt(y[0])), 0.0), (1 / (2 * math.sqrt(y[0])), -1 / (2 * math.sqrt(y[1]))))

    def Fu(self, y, x):
        return (tuple(self.P["c"]), (0.0, 0.0, 0.0))

    def G(self, y, x):
        return self.P["k1"] * (y[1] - self.P["k2"]) ** 2

    def Gy(self, y, x):
        return (0.0, 2 * self.P["k1"] * (y[1] - self.P["k2"]))


class _VanDerPol:
    """example_vanderpol.jl:48-81."""
    P = VANDERPOL

    def F(self, y, x):
        s = _sum3(self.P["c"], x)
        return (y[1], (1 - y[0] ** 2) * y[1] * s - y[0])

    def Fy(self, y, x):
        s = _sum3(self.P["c"], x)
        return ((0.0, 1.0), (-2 * y[0] * y[1] * s - 1, (1 - y[0] ** 2) * s))

    def Fu(self, y, x):
        # [0 0 0; c' * (1 - y1^2) * y2]: the row c' scaled by (1 - y1^2), then by y2
        return ((0.0, 0.0, 0.0), tuple((c * (1 - y[0] ** 2)) * y[1] for c in self.P["c"]))

    def G(self, y, x):
        return y[0] ** 2 + y[1] ** 2

    def Gy(self, y, x):
        return (2 * y[0], 2 * y[1])


PROBLEMS = {"fishing": _Fishing, "doubletank": _DoubleTank, "vanderpol": _VanDerPol}


class ODEOracle:
    """eval_f / eval_df of one example for a control x given as nt columns of 3 floats (x[i] = x[:, i+1])."""

    def __init__(self, name, nt):
        self.h = PROBLEMS[name]()
        self.nt = int(nt)
        self.T0, self.T1 = self.h.P["T0"], self.h.P["T1"]
        self.tau = (self.T1 - self.T0) / self.nt  # tau = (T1 - T0) / nt (example structs)
        self.state0 = tuple(self.h.P["state0"])

    def eval_f(self, x, keep_states=False):
        """ODEObjective.jl:125-150; x: sequence of nt control columns."""
        h, tau, nt = self.h, self.tau, self.nt
        y = self.state0
        fval = 0.5 * h.G(self.state0, x[0])
        states = []
        for i in range(nt):
            f = h.F(y, x[i])
            y = (y[0] + tau * f[0], y[1] + tau * f[1])  # @. state += tau * Fval
            states.append(y)
            if i < nt - 1:
                fval += h.G(y, x[i + 1])
            else:
                fval += 0.5 * h.G(y, x[nt - 1])
        fval *= tau
        return (fval, states) if keep_states else fval

    def eval_df(self, x):
        """ODEObjective.jl:153-184 after eval_f at the same x; returns (J, df) with df[i] the column of step i."""
        h, tau, nt = self.h, self.tau, self.nt
        J, st = self.eval_f(x, keep_states=True)
        adj = [None] * nt
        g = h.Gy(st[nt - 1], x[nt - 1])
        adj[nt - 1] = (-0.5 * tau * g[0], -0.5 * tau * g[1])
        for i in range(nt - 1, 0, -1):  # Julia i = nt-1:-1:1; state[:, i] -> st[i-1], x[:, i+1] -> x[i]
            g = h.Gy(st[i - 1], x[i])
            fy = h.Fy(st[i - 1], x[i])
            a = adj[i]
            fta = (fy[0][0] * a[0] + fy[1][0] * a[1], fy[0][1] * a[0] + fy[1][1] * a[1])  # Fyval' * adjoint
            adj[i - 1] = (a[0] + tau * (fta[0] - g[0]), a[1] + tau * (fta[1] - g[1]))
        df = []
        for i in range(nt):  # Julia i = 1:nt; state = state0 at i = 1 else state[:, i-1]
            y = self.state0 if i == 0 else st[i - 1]
            fu = h.Fu(y, x[i])
            a = adj[i]
            df.append(tuple((0.0 - (fu[0][m] * a[0] + fu[1][m] * a[1])) + 0.0 for m in range(3)))  # Gu = 0
        return J, df

    def fd_check(self, x, hdir, t=1e-6):
        """The reference's test_df (example_fishing.jl:94-123): |(f(x + t h) - f(x)) / t - tau sum_i df_i' h_i|."""
        J, df = self.eval_df(x)
        dfh = 0.0
        for i in range(self.nt):
            dfh += self.tau * sum(df[i][m] * hdir[i][m] for m in range(3))
        xt = [tuple(x[i][m] + t * hdir[i][m] for m in range(3)) for i in range(self.nt)]
        return abs((self.eval_f(xt) - J) / t - dfh), abs(dfh)
