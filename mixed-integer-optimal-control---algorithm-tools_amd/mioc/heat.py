"""The PDE heat objective: host-side problem data + the device gradient producer.

Reference: julia_opt/example_heat.jl (HeatObj: ∂ₜy − αΔy = f₁u₁ + f₂u₂ on [-1,1]² × [0,10], ∂y/∂n + κy = κ·Tout,
two Gaussian heaters, G = ½‖y − yd‖²_M, G_t = γ·Σu) over julia_opt/PDEObjective.jl:129-199 (implicit Euler state and
adjoint with the precomputed LU factors, trapezoid cost, df = (M⁻¹F)ᵀp + Gu).

The reference assembles A, M, F and state0 with its FEM bundle (julia_fem/: a Triangle mesh of the square refined
three times, P2 Lagrange elements).  That assembly is the caller's, outside the hot path: the C ABI takes the
assembled matrices (``mioc_heat_setup``).  ``HeatProblem`` here is a stand-in with the same structure for tests and
the bench -- P1 elements on a structured n x n grid of the square (n = 17 gives N = 289 degrees of freedom, the
P2 count of a 9 x 9 vertex grid) with the same coefficients, heaters, Robin boundary and targets -- not the
reference's mesh.  The time loops, the cost and the gradient (the part the reference spends its time in) run on the
device and are checked against the oracle's LU restatement (oracle/heat_oracle.py) on the same matrices.
"""
from __future__ import annotations

import numpy as np

from .iterators import product_iterator
from .objective import AbstractObjectiveLazy


class HeatProblem:
    """Assembled data of example_heat.jl:23-116 on a structured P1 mesh (a stand-in for FEMBundle's P2 mesh)."""

    def __init__(self, n=17, nt=500, T0=0.0, T1=10.0, alpha=1.0, c1=(10.0, 10.0), c2=(20.0, 20.0), kappa=0.12,
                 Tout=0.0, temp0=10.0, tempT=20.0, gamma=10.0, heaters=((-1.0, 0.0), (1.0, 0.0))):
        self.n, self.nt, self.T0, self.T1, self.gamma = n, nt, T0, T1, gamma
        self.tau = (T1 - T0) / nt  # example_heat.jl:90
        self.levels = [list(range(6)), list(range(6))]  # 𝓥 = [[0..5], [0..5]] (example_heat.jl:42)
        xs = np.linspace(-1.0, 1.0, n)
        P = np.array([(xs[i], xs[j]) for j in range(n) for i in range(n)])
        N = n * n
        tris = []
        for j in range(n - 1):
            for i in range(n - 1):
                v00, v10, v01, v11 = i + n * j, i + 1 + n * j, i + n * (j + 1), i + 1 + n * (j + 1)
                tris += [(v00, v10, v11), (v00, v11, v01)]
        A = np.zeros((N, N))
        M = np.zeros((N, N))
        F = np.zeros((N, len(heaters)))
        rhs = [lambda x, q=q: c2[q] * np.exp(-c1[q] * ((x[0] - heaters[q][0]) ** 2 + (x[1] - heaters[q][1]) ** 2))
               for q in range(len(heaters))]
        for t in tris:
            p = P[list(t)]
            d = np.array([[p[1, 0] - p[0, 0], p[2, 0] - p[0, 0]], [p[1, 1] - p[0, 1], p[2, 1] - p[0, 1]]])
            area = 0.5 * abs(np.linalg.det(d))
            g = np.linalg.solve(d.T, np.array([[-1.0, 1.0, 0.0], [-1.0, 0.0, 1.0]]))  # ∇φ of the 3 vertices
            Ke = alpha * area * (g.T @ g)
            Me = area / 12.0 * (np.ones((3, 3)) + np.eye(3))
            mids = [(p[a] + p[b]) / 2 for a, b in ((0, 1), (1, 2), (2, 0))]  # edge-midpoint rule (exact for P2)
            phi = np.array([[0.5, 0.0, 0.5], [0.5, 0.5, 0.0], [0.0, 0.5, 0.5]])  # φ_a(mid_m) as [a][m]
            for a in range(3):
                for b in range(3):
                    A[t[a], t[b]] += Ke[a, b]
                    M[t[a], t[b]] += Me[a, b]
                for q in range(len(heaters)):
                    F[t[a], q] += area / 3.0 * sum(rhs[q](mids[m]) * phi[a, m] for m in range(3))
        # Robin boundary: κ∫_Γ φ_a φ_b into A, κ·Tout ∫_Γ φ_a into every column of F (assemble_rhs adds G to each)
        bnd = []
        for i in range(n - 1):
            bnd += [(i, i + 1), (i + n * (n - 1), i + 1 + n * (n - 1)), (n * i, n * (i + 1)),
                    (n - 1 + n * i, n - 1 + n * (i + 1))]
        for a, b in bnd:
            ln = float(np.linalg.norm(P[a] - P[b]))
            A[a, a] += kappa * ln / 3.0
            A[b, b] += kappa * ln / 3.0
            A[a, b] += kappa * ln / 6.0
            A[b, a] += kappa * ln / 6.0
            F[a, :] += kappa * Tout * ln / 2.0
            F[b, :] += kappa * Tout * ln / 2.0
        self.N, self.A, self.M, self.F = N, A, M, F
        Lc = np.linalg.cholesky(M)  # calculate_M_invA / _invF use cholesky(M) (example_heat.jl:242-262)
        solve = lambda B: np.linalg.solve(Lc.T, np.linalg.solve(Lc, B))  # noqa: E731
        self.M_invA = solve(A)
        self.M_invF = solve(F)
        self.state0 = np.linalg.solve(M, M @ np.full(N, temp0))  # assemble_state0: M \ ∫ y0 φ
        self.yd = np.full((N, nt + 1), tempT)  # assemble_yd

    def setup(self, ctx):
        """Hand the matrices to a native.Context (mioc_heat_setup)."""
        ctx.heat_setup(self.M_invA, self.M_invF, self.M, self.state0, self.yd, self.T0, self.T1, self.gamma)


class HeatObj(AbstractObjectiveLazy):
    """The reference's HeatObj (example_heat.jl:23-116) as a lazy objective for TRM: eval_f_helper and
    eval_df_helper (PDEObjective.jl:142-199) run on the device through mioc_heat_eval (no CPU path).  One
    device call computes both; the gradient of the last eval_f at obj.x is kept and handed out by eval_df."""

    def __init__(self, problem=None, ctx=None, device=0, **kw):
        from .native import Context
        self.problem = HeatProblem(**kw) if problem is None else problem
        hp = self.problem
        self.T0, self.T1, self.nt, self.tau, self.gamma = hp.T0, hp.T1, hp.nt, hp.tau, hp.gamma
        self.V = [list(v) for v in hp.levels]
        self.iterator = product_iterator(self.V)  # no restrictions on the integer controls (example_heat.jl:44)
        self.nu, self.nv = 0, len(self.V)
        self.nx = self.nu + self.nv
        self._init_fields(self.nx, self.nt)
        self.ctx = Context(device) if ctx is None else ctx
        hp.setup(self.ctx)
        self._df_at = None

    def eval_f_helper(self, x, cache):
        J, df = self.ctx.heat_eval(np.asarray(x, dtype=np.float64)[None])
        if cache:
            self._df_at = (np.array(x, copy=True), df[0])
        return float(J[0])

    def eval_df_helper(self):
        if self._df_at is None or not np.array_equal(self._df_at[0], self.x):
            _, df = self.ctx.heat_eval(np.asarray(self.x, dtype=np.float64)[None])
            self._df_at = (np.array(self.x, copy=True), df[0])
        self.df[:, :] = self._df_at[1]
