"""Multi-start TRM with every restart's data on the device.

The control flow is multi-trust.jl:53-170 per restart, run for K restarts in lock step:

  outer iteration   TV_old = TV_p(u), ∇f = eval_df!(u)                       multi-trust.jl:99-103
  inner iteration   bellman_TRM! (first) or eval_u_TRM! at B_new (halved)    :108-114
                    int_val, TV_new, pred                                     :117-126  (mioc_pred_batch_device)
                    J_new = eval_f!(u), ared, stop / halve / accept           :124-158  (mioc_trm_decide_device)
  return            J + β·TV_p(u)                                            :169

Device kernels do all O(nt) work: the random starts (mioc_rand_start_device, HelpFunctions.jl:204-225), the ODE
objective and adjoint gradient (mioc_ode_eval_device, ODEObjective.jl:125-184) or the PDE heat objective's
(mioc_heat_eval_device, PDEObjective.jl:129-199), the DP and backtrack with one budget
per restart after halving (mioc_backtrack_batch_budgets_device), pred and TV_p, and the decision.  Per inner
iteration the host reads back K decision codes and keeps K small counters (Δᵏ, k, flags); the controls never leave
HBM.  The context enqueues on its own stream and the few torch element-wise updates (masks, where) run on
torch's, so every hand-over between the two is synchronised (`_to_torch` / `_to_ctx`).  Restarts that left their
inner loop wait for the others (their lanes of a batched call are ignored), so every
restart follows exactly the sequence of the single-restart loop, including its quirks: the gradient of the next
outer iteration is taken at the last trial u (obj.x), accepted or not, and a stop returns J_old + β·TV_p(u_trial).
"""
from __future__ import annotations

import math

import numpy as np

from .iterators import LevelTable, bounded_sum_iterator
from .native import (MIOC_ODE_DOUBLETANK, MIOC_ODE_FISHING, MIOC_ODE_VANDERPOL, Context)

# the reference's ODE examples: (problem code, default nt, T0, T1) -- example_fishing.jl, example_doubletank.jl,
# example_vanderpol.jl; all three are SOS1 over three binary controls
PROBLEMS = {"fishing": (MIOC_ODE_FISHING, 1200, 0.0, 12.0), "doubletank": (MIOC_ODE_DOUBLETANK, 1000, 0.0, 10.0),
            "vanderpol": (MIOC_ODE_VANDERPOL, 2000, 0.0, 20.0)}


def sos1_levels():
    V = [[0, 1], [0, 1], [0, 1]]
    return LevelTable(V, bounded_sum_iterator(V, 1, 1))


def TRM_batch(problem, par, K=None, x0=None, seed=0, nt=None, device=0, log=None):  # noqa: C901
    """Run TRM (multi-trust.jl:53-170) for K restarts of an ODE example, or of the PDE heat example, on the device.

    problem: "fishing" / "doubletank" / "vanderpol", or a mioc.heat.HeatProblem (example_heat.jl: 6 x 6 product
    levels, gradient from mioc_heat_eval_device; its nt is the problem's).
    x0: a (K, nt, nx) float64 CUDA tensor of starts, or None for K device random starts (rand_func_int with `seed`).
    Returns (values (K,) numpy: J + β·TV_p(u) per restart, u (K, nt, nx) CUDA tensor: obj.x of each restart,
    iterations (K,) numpy)."""
    import torch

    ctx = Context(device)
    if isinstance(problem, str):
        prob, nt_def, T0, T1 = PROBLEMS[problem]
        lt = sos1_levels()

        def evalf(x, J, df):
            ctx.ode_eval_tensors(prob, x, T0, T1, J, df)
    else:  # the PDE heat objective (PDEObjective.jl:129-199, example_heat.jl)
        hp = problem
        nt_def, T0, T1 = hp.nt, hp.T0, hp.T1
        if nt is not None and int(nt) != hp.nt:
            raise ValueError("the heat problem fixes nt")
        lt = LevelTable(hp.levels)
        hp.setup(ctx)

        def evalf(x, J, df):
            ctx.heat_eval_tensors(x, J, df)

    def _to_torch():  # the context's results are read by torch ops
        ctx.synchronize()

    def _to_ctx():  # torch's writes are read by the context's stream
        torch.cuda.current_stream(dev).synchronize()

    ctx.set_levels(lt)
    ctx.set_cost(par.p, par.beta)
    dev = torch.device("cuda", device)
    if x0 is None:
        nt = nt_def if nt is None else int(nt)
        u = torch.empty(int(K), nt, lt.M, dtype=torch.float64, device=dev)
        ctx.rand_start_tensor(u, seed)
    else:
        u = x0.to(device=dev, dtype=torch.float64).contiguous().clone()
    K, nt, _ = u.shape
    _to_torch()
    tau = (T1 - T0) / nt
    beta, D0, sigma, kmax, maxiter = par.beta, par.Delta0, par.sigma, par.kmax, par.maxiter
    B = int(math.floor(D0 / tau))  # multi-trust.jl:69

    f64 = dict(dtype=torch.float64, device=dev)
    u_old = u.clone()
    J_old = torch.empty(K, **f64)
    _to_ctx()
    evalf(u, J_old, None)
    tv_u = torch.empty(K, **f64)
    ctx.tv_tensors(u, tv_u)               # TV of the current u; afterwards every trial's TV_new
    J = torch.full((K,), math.inf, **f64)
    df = torch.empty_like(u)
    trial = torch.empty_like(u)
    int_val, tv_o, tv_new, pred = (torch.empty(K, **f64) for _ in range(4))
    J_new = torch.empty(K, **f64)
    dec = torch.empty(K, dtype=torch.int32, device=dev)
    budgets = torch.empty(K, dtype=torch.int32, device=dev)
    stop = np.zeros(K, dtype=bool)
    iters = np.zeros(K, dtype=np.int64)
    _to_torch()
    _to_ctx()
    it = 1
    while not stop.all() and it <= maxiter:
        active = ~stop
        _to_torch()
        TV_old = tv_u.clone()                                    # TV_p(u, p), multi-trust.jl:99
        _to_ctx()
        evalf(u, None, df)                                       # ∇f at obj.x = u, :102-103
        ctx.bellman_batch_tensors(df, u_old, B, tau)
        Dk = np.full(K, D0)
        k = np.ones(K, dtype=np.int64)
        inner = active.copy()                                    # restarts still inside the inner loop
        halved = np.zeros(K, dtype=bool)
        while inner.any():
            Bk = np.where(halved, np.floor(Dk / tau), B).astype(np.int32)  # B_new = floor(Δᵏ/Δt), :109
            budgets.copy_(torch.from_numpy(Bk))
            _to_ctx()
            ctx.backtrack_batch_budgets_tensors(budgets, trial)
            ctx.pred_batch_tensors(int_val, tv_o, tv_new, pred)
            _to_torch()
            # pred with TV_old = TV_p(u) of the outer iteration (the device's tv_o is TV_p(u_old); they differ
            # after an inner loop that ran out of kmax, where u is a rejected trial)
            pred_ref = int_val + beta * (TV_old - tv_new)
            _to_ctx()
            evalf(trial, J_new, None)
            ctx.trm_decide_tensors(J_old, J_new, TV_old, tv_new, pred_ref, sigma, dec)
            ctx.synchronize()
            d = dec.cpu().numpy()
            m = torch.from_numpy(inner).to(dev)
            u[m] = trial[m]                                      # obj.x = the trial, accepted or not
            tv_u = torch.where(m, tv_new, tv_u)
            if log is not None:
                log.append((it, k.copy(), Dk.copy(), pred_ref.cpu().numpy(), d.copy(), inner.copy()))
            st = inner & (d == 2)                                # pred <= 0: stop, J = J_old, :130-138
            acc = inner & (d == 0)                               # good step, :148-154
            bad = inner & (d == 1)                               # Δᵏ halved, :140-146
            if st.any():
                ms = torch.from_numpy(st).to(dev)
                J = torch.where(ms, J_old, J)
                stop |= st
            if acc.any():
                ma = torch.from_numpy(acc).to(dev)
                u_old[ma] = trial[ma]
                J_old = torch.where(ma, J_new, J_old)
                J = torch.where(ma, J_new, J)
                TV_old = torch.where(ma, tv_new, TV_old)
            Dk = np.where(bad, Dk / 2, Dk)
            halved |= bad
            k = np.where(inner, k + 1, k)
            inner = inner & ~st & ~acc & (k <= kmax)
            _to_ctx()
        iters[active] += 1
        it += 1
    _to_ctx()
    evalf(u, None, df)                                           # final derivative, :166-167
    _to_torch()
    values = (J + beta * tv_u).cpu().numpy()                     # J + β·TV_p(u, p), :169
    ctx.close()
    return values, u, iters
