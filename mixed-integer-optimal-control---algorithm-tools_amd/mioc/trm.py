"""The trust-region driver ``TRM`` and the subproblem entry points, over the HIP library.

Mirrors the reference:
  TRM_parameters                  multi-trust.jl:26-34
  TRM(obj, par; x0)               multi-trust.jl:53-170
  bellman_TRM! / eval_u_TRM!      HelpFunctions.jl:20-83 / :98-124  (run on the GPU via libmioc)
  TV_p                            HelpFunctions.jl:251-273
  rand_func / rand_func_int       HelpFunctions.jl:136-148 / :204-225

Differences that are deliberate and documented:
  * U and Φ live in device memory owned by a ``SubproblemSolver``; there is no host U/Φ
    (the reference's Int64 U would be 2.21 TB at nt=65536, 4096 levels, B=256);
  * the default start uses numpy's PCG64 instead of Julia's MersenneTwister + StatsBase.sample, so
    pass ``x0`` explicitly for reproducible runs (the reference's default is random too).
"""
from __future__ import annotations

import math

import numpy as np

from .iterators import LevelTable
from .native import Context, MiocNativeError
from .objective import eval_df_, eval_f_


class TRM_parameters:
    """Algorithmic parameters (multi-trust.jl:26-34).  Greek keyword aliases are accepted."""

    def __init__(self, beta=0.001, p=1, Delta0=1.0, sigma=0.5, kmax=40, maxiter=1000, log=False, **kw):
        alias = {"β": "beta", "Δ⁰": "Delta0", "Δ0": "Delta0", "σ": "sigma"}
        vals = dict(beta=beta, p=p, Delta0=Delta0, sigma=sigma, kmax=kmax, maxiter=maxiter, log=log)
        for k, v in kw.items():
            if k not in alias:
                raise TypeError(f"unknown TRM parameter {k!r}")
            vals[alias[k]] = v
        self.beta = float(vals["beta"])
        self.p = vals["p"]
        self.Delta0 = float(vals["Delta0"])
        self.sigma = float(vals["sigma"])
        self.kmax = int(vals["kmax"])
        self.maxiter = int(vals["maxiter"])
        self.log = bool(vals["log"])

    def __repr__(self):
        return (f"TRM_parameters(beta={self.beta}, p={self.p}, Delta0={self.Delta0}, sigma={self.sigma}, "
                f"kmax={self.kmax}, maxiter={self.maxiter}, log={self.log})")


def TV_p(u, p):
    """sum_i ||u_i - u_{i-1}||_p; p = Inf is the max-norm (HelpFunctions.jl:251-268).  None -> 0."""
    if u is None:
        return 0.0
    u = np.asarray(u, dtype=np.float64)
    d = np.abs(np.diff(u, axis=1))
    if p == math.inf:
        val = 0.0
        for s in d.max(axis=0) if d.size else []:
            val += float(s)
        return val
    if p > 0:
        val = 0.0
        for i in range(d.shape[1]):
            s = 0.0
            for m in range(d.shape[0]):
                s += float(d[m, i]) ** p
            val += s ** (1.0 / p)
        return val
    raise ValueError("Only positive integer valued `p` are accepted!")


class SubproblemSolver:
    """Owns one device context and keeps the DP of the last ``bellman`` resident.

    ``bellman(df, u_old, B, dt)`` is bellman_TRM!; ``backtrack(B_use)`` is eval_u_TRM! and may be
    called repeatedly with smaller budgets (the halving path, multi-trust.jl:108-110).
    """

    def __init__(self, levels: LevelTable, p, beta, device=0, table=None):
        self.levels = levels
        self.ctx = Context(device)
        self.ctx.set_levels(levels)
        self.ctx.set_cost(p, beta, table=table)

    def bellman(self, df, u_old, B, dt):
        self.ctx.bellman(df, u_old, B, dt)

    def backtrack(self, B_use):
        u, phi, _sw = self.ctx.backtrack(B_use)
        return u, phi

    def pred(self):
        """(int_val, TV_p(u_old), TV_p(u), pred) of the last backtrack, reduced on the device
        (multi-trust.jl:117-126; mioc_pred)."""
        return self.ctx.pred()


def bellman_TRM_(solver, df, u_old, B, dt):
    """bellman_TRM!(∇f, u_old, B, β, p, Δt, nu, U, Φ, iterator) -- U/Φ are the solver's device state."""
    solver.bellman(df, u_old, B, dt)


def eval_u_TRM_(solver, u, u_old, B):
    """eval_u_TRM!(u, u_old, U, Φ, B, nu): fills ``u`` in place, returns Φ*."""
    un, phi = solver.backtrack(B)
    u[:, :] = un
    return phi


def rand_func_int(obj, rng=None, jumps=None):
    """Piecewise-constant admissible start (HelpFunctions.jl:204-225) -- numpy PCG64, not Julia's MT."""
    g = np.random.default_rng(rng)
    nt = int(obj.nt)
    jumps = nt // 10 if jumps is None else int(jumps)
    tuples = [tuple(t) for t in obj.iterator]
    t = np.sort(g.choice(np.arange(2, nt + 1), size=min(jumps, nt - 1), replace=False))
    v0 = np.zeros((len(obj.V), nt), dtype=np.float64)
    j = 0
    l = tuples[g.integers(len(tuples))]
    for i in range(1, nt + 1):
        if j < len(t) and i >= t[j]:
            j += 1
            l = tuples[g.integers(len(tuples))]
        v0[:, i - 1] = [obj.V[m][l[m] - 1] for m in range(len(obj.V))]
    return v0


def rand_func(obj, rng=None, jumps=None):
    """Random admissible control x0 (HelpFunctions.jl:136-148); integer part only (nu = 0 here)."""
    x0 = np.zeros((obj.nx, obj.nt), dtype=np.float64, order="F")
    x0[obj.nx - len(obj.V):, :] = rand_func_int(obj, rng=rng, jumps=jumps)
    return x0


def TRM(obj, par=None, x0=None, solver=None, device=0, rng=None):
    """Trust-region method with Bellman subproblems (multi-trust.jl:53-170).

    Returns J + β·TV_p(u, p) exactly as the reference does (:169), including its quirks: on
    pred <= 0 it returns J_old + β·TV_p(u_trial) while obj.x holds the rejected trial (:130-138).
    ``solver`` defaults to a ``SubproblemSolver`` on HIP device ``device`` (no CPU fallback).
    """
    par = TRM_parameters() if par is None else par
    n = int(obj.nt)
    dt = float(obj.tau)
    beta, D0, sigma, p, kmax, maxiter = par.beta, par.Delta0, par.sigma, par.p, par.kmax, par.maxiter
    if solver is None:
        solver = SubproblemSolver(LevelTable(obj.V, obj.iterator), p, beta, device=device)
    u = obj.x
    u[:, :] = rand_func(obj, rng=rng) if x0 is None else x0
    u_old = np.array(u, dtype=np.float64, order="F", copy=True)
    B = int(math.floor(D0 / dt))

    J = math.inf
    it = 1
    stop = False
    J_old = eval_f_(obj)
    tv_u = TV_p(u, p)  # TV of the current u; afterwards every trial's TV_new from the device
    if par.log:
        print(" Iter |   k |   Δᵏ   |      J      |   pred   |   ared   |       step            ")
        print("-" * 81)
        print(f"{0:5d} |{0:4d} | {D0:6.2f} | {J_old + beta * tv_u:.5e} | {0.0:8.4f} | {0.0:8.4f} | "
              f"Initial Value   ")
    while not stop and it <= maxiter:
        Dk = D0
        k = 1
        ared = 0.0
        pred = 1.0
        halved = False
        TV_old = tv_u  # TV_p(u, p) (multi-trust.jl:99): u is the last trial or the accepted control
        eval_df_(obj)
        grad = obj.df
        while ared < sigma * pred and k <= kmax:
            if halved:
                B_new = int(math.floor(Dk / dt))
                eval_u_TRM_(solver, u, u_old, B_new)
            else:
                bellman_TRM_(solver, grad, u_old, B, dt)
                eval_u_TRM_(solver, u, u_old, B)
            # int_val = Δt Σ_j ∇f_j'(u_old_j - u_j) and TV_new = TV_p(u, p): O(nt) reductions on the device
            int_val, _tv_uold, TV_new, _ = solver.pred()
            tv_u = TV_new
            J_new = eval_f_(obj)
            pred = int_val + beta * (TV_old - TV_new)
            ared = J_old - J_new + beta * (TV_old - TV_new)
            if pred <= 0:
                J = J_old
                stop = True
                if par.log:
                    print(f"{it:5d} |{k:4d} | {Dk:6.2f} | {J + beta * TV_old:.5e} | {pred:8.4f} | {ared:8.4f} | "
                          f"optimal solution found   ")
                break
            elif ared < sigma * pred:
                if par.log:
                    print(f"{it:5d} |{k:4d} | {Dk:6.2f} | {J_old + beta * TV_old:.5e} | {pred:8.4f} | "
                          f"{ared:8.4f} | bad step, Δᵏ halved   ")
                Dk = Dk / 2
                halved = True
            else:
                u_old[:, :] = u
                J_old = J_new
                TV_old = TV_new
                J = J_new
                if par.log:
                    print(f"{it:5d} |{k:4d} | {Dk:6.2f} | {J + beta * TV_new:.5e} | {pred:8.4f} | {ared:8.4f} | "
                          f"good step   ")
            k += 1
        it += 1
    eval_df_(obj)
    return J + beta * tv_u


__all__ = ["TRM_parameters", "TRM", "TV_p", "SubproblemSolver", "bellman_TRM_", "eval_u_TRM_", "rand_func",
           "rand_func_int", "MiocNativeError"]
