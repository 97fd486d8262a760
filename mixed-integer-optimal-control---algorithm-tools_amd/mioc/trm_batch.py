"""Multi-start TRM with every restart's data and its control state on the device.

The control flow is multi-trust.jl:53-170 per restart, run for K restarts in lock step:

  outer iteration   TV_old = TV_p(u), ∇f = eval_df!(u)                       multi-trust.jl:99-103
  inner iteration   bellman_TRM! (first) or eval_u_TRM! at B_new (halved)    :108-114
                    int_val, TV_new                                           :117-126  (mioc_pred_batch_device)
                    J_new = eval_f!(u), pred, ared, stop / halve / accept     :124-158  (mioc_trm_inner_end_device)
  return            J + β·TV_p(u)                                            :169

Device kernels do all O(nt) work: the random starts (mioc_rand_start_device, HelpFunctions.jl:204-225), the ODE
objective and adjoint gradient (mioc_ode_eval_device, ODEObjective.jl:125-184) or the PDE heat objective's
(mioc_heat_eval_device, PDEObjective.jl:129-199), the DP and backtrack with one budget per restart after halving
(mioc_backtrack_batch_budgets_device), pred and TV_p -- and the control itself: Δᵏ, k, the inner / halved / stopped
flags, the decision, obj.x = trial, the accept bookkeeping and the next budgets live in a device state block
(mioc_trm_outer_begin_device / mioc_trm_inner_end_device).  Everything is enqueued on the context's stream; the
host enqueues inner iterations in chunks and reads back two flags (any restart still in its inner loop, any restart
not stopped) once per chunk (mioc_trm_poll) -- with the default chunk of 2 that is one read-back per outer
iteration whenever every inner loop ends within two trials.  Kernels of an inner iteration that no restart needs
return at once (the state's gate word, mioc_trm_attach).  Restarts that left their inner loop are ignored by the
state update, so every restart follows exactly the sequence of the single-restart loop, including its quirks: the
gradient of the next outer iteration is taken at the last trial u (obj.x), accepted or not, and a stop returns
J_old + β·TV_p(u_trial).
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


def TRM_batch(problem, par, K=None, x0=None, seed=0, nt=None, device=0, log=None, inner_chunk=2,  # noqa: C901
              stats=None):
    """Run TRM (multi-trust.jl:53-170) for K restarts of an ODE example, or of the PDE heat example, on the device.

    problem: "fishing" / "doubletank" / "vanderpol", or a mioc.heat.HeatProblem (example_heat.jl: 6 x 6 product
    levels, gradient from mioc_heat_eval_device; its nt is the problem's).
    x0: a (K, nt, nx) float64 CUDA tensor of starts, or None for K device random starts (rand_func_int with `seed`).
    log: a list to receive (inner iteration, decisions (K,)) after every inner iteration (debugging: one stream
    synchronisation each).  inner_chunk: inner iterations enqueued between two read-backs of the control flags.
    stats: a dict to receive {"polls": read-backs, "outer": outer iterations}.
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
    tau = (T1 - T0) / nt
    beta, D0, sigma, kmax, maxiter = par.beta, par.Delta0, par.sigma, par.kmax, par.maxiter
    B = int(math.floor(D0 / tau))  # multi-trust.jl:69

    f64 = dict(dtype=torch.float64, device=dev)
    _to_torch()                            # u (random starts) from the context's stream
    u_old = u.clone()
    J_old = torch.empty(K, **f64)
    tv_u = torch.empty(K, **f64)
    J = torch.full((K,), math.inf, **f64)
    df = torch.empty_like(u)
    trial = torch.empty_like(u)
    int_val, tv_o, tv_new, pred = (torch.empty(K, **f64) for _ in range(4))
    J_new = torch.empty(K, **f64)
    dec = torch.empty(K, dtype=torch.int32, device=dev)
    budgets = torch.empty(K, dtype=torch.int32, device=dev)
    state = ctx.trm_state_tensor(K)
    _to_ctx()                              # every buffer above (torch's stream) before the context's stream
    evalf(u, J_old, None)
    ctx.tv_tensors(u, tv_u)                # TV of the current u; afterwards every trial's TV_new
    ctx.trm_attach(state)
    polls = 0
    try:
        it = 1
        while it <= maxiter:
            ctx.trm_outer_begin(state, tv_u, D0, B, budgets)         # TV_old, Δᵏ, k, inner, :99-107
            evalf(u, None, df)                                      # ∇f at obj.x = u, :102-103
            ctx.bellman_batch_tensors(df, u_old, B, tau)
            done, active = 0, True
            while done < kmax:
                for _ in range(min(inner_chunk, kmax - done)):
                    ctx.backtrack_batch_budgets_tensors(budgets, trial)
                    ctx.pred_batch_tensors(int_val, tv_o, tv_new, pred)
                    evalf(trial, J_new, None)
                    ctx.trm_inner_end(state, sigma, kmax, tau, B, int_val, tv_new, J_new, J_old, J, tv_u, budgets,
                                      trial, u, u_old, decision=dec if log is not None else None)
                    done += 1
                    if log is not None:                             # debugging: one synchronisation per trial
                        st = ctx.trm_state_arrays(state, K)
                        d = dec.cpu().numpy().copy()
                        log.append((it, st["k"].copy(), st["Dk"].copy(), None, d, d >= 0))
                inner, active = ctx.trm_poll(state)                  # the one read-back per chunk
                polls += 1
                if not inner:
                    break
            it += 1
            if not active:                                          # every restart stopped, :96
                break
    finally:
        ctx.trm_attach(None)
    evalf(u, None, df)                                              # final derivative, :166-167
    _to_torch()
    values = (J + beta * tv_u).cpu().numpy()                        # J + β·TV_p(u, p), :169
    st = ctx.trm_state_arrays(state, K)
    iters = st["iters"].astype(np.int64)
    if stats is not None:
        stats.update(polls=polls, outer=it - 1)
    ctx.close()
    return values, u, iters
