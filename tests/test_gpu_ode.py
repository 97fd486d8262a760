"""GPU parity of the batched ODE gradient producer: mioc_ode_eval_device against the host mirror
of julia_opt/ODEObjective.jl:125-184 with the fishing / doubletank / vanderpol hooks (mioc/ode.py).

Bar: J and df within 1e-12 relative of the mirror (the mirror's numpy small dot / matvec may round in another
order or through BLAS; the device sums left to right without FMA), and a whole batched trust-region iteration
(gradient -> DP -> backtrack -> pred) on the device equal to the host path fed the same gradient.
"""
import math

import numpy as np
import pytest

import mioc
from mioc import native
from mioc.iterators import LevelTable

pytestmark = pytest.mark.gpu

CASES = [("fishing", native.MIOC_ODE_FISHING, 512), ("doubletank", native.MIOC_ODE_DOUBLETANK, 1000),
         ("vanderpol", native.MIOC_ODE_VANDERPOL, 2000)]


def _obj(name, nt):
    from mioc.ode import DTMObj, LVMObj, VPOObj
    return {"fishing": LVMObj, "doubletank": DTMObj, "vanderpol": VPOObj}[name](nt=nt)


@pytest.mark.parametrize("name,prob,nt", CASES, ids=[c[0] for c in CASES])
def test_ode_eval_vs_host_mirror(name, prob, nt):
    import torch
    K = 16
    obj = _obj(name, nt)
    xs = [mioc.rand_func(obj, rng=100 + k) for k in range(K)]
    Jh, dfh = [], []
    for x in xs:
        obj.x[:, :] = x
        Jh.append(mioc.eval_f_(obj))
        mioc.eval_df_(obj)
        dfh.append(np.array(obj.df, copy=True))
    ctx = native.Context(0)
    dx = torch.tensor(np.ascontiguousarray(np.stack([x.T for x in xs])), dtype=torch.float64, device="cuda")
    J = torch.empty(K, dtype=torch.float64, device="cuda")
    df = torch.empty_like(dx)
    ctx.ode_eval_tensors(prob, dx, obj.T0, obj.T1, J, df)
    ctx.synchronize()
    J, df = J.cpu().numpy(), df.cpu().numpy()
    exact = 0
    for k in range(K):
        assert abs(J[k] - Jh[k]) <= 1e-12 * abs(Jh[k]), (k, J[k], Jh[k])
        d, h = df[k].T, dfh[k]
        assert np.max(np.abs(d - h)) <= 1e-12 * max(1e-300, np.max(np.abs(h))), k
        exact += int(J[k] == Jh[k]) + int(np.array_equal(d, h))
    print(f"{name}: {exact} of {2 * K} J / df arrays bit-identical to the host mirror")
    ctx.close()


def test_device_trust_region_iteration_equals_host():
    """One trust-region inner iteration for K fishing restarts entirely on the device (gradient, bellman_TRM!,
    eval_u_TRM!, pred, and J at the trial) against the host TRM pieces on the same controls."""
    import torch
    K, nt = 32, 256
    obj = _obj("fishing", nt)
    lt = LevelTable(obj.V, obj.iterator)
    par = mioc.TRM_parameters(beta=1e-4, Delta0=2, p=math.inf)
    B = int(math.floor(par.Delta0 / obj.tau))
    xs = [mioc.rand_func(obj, rng=7 + k) for k in range(K)]
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(par.p, par.beta)
    dx = torch.tensor(np.ascontiguousarray(np.stack([x.T for x in xs])), dtype=torch.float64, device="cuda")
    Jold = torch.empty(K, dtype=torch.float64, device="cuda")
    df = torch.empty_like(dx)
    ctx.ode_eval_tensors(native.MIOC_ODE_FISHING, dx, obj.T0, obj.T1, Jold, df)
    ctx.bellman_batch_tensors(df, dx, B, obj.tau)
    du = torch.empty_like(dx)
    ctx.backtrack_batch_tensors(B, du)
    outs = [torch.empty(K, dtype=torch.float64, device="cuda") for _ in range(4)]
    ctx.pred_batch_tensors(*outs)
    Jnew = torch.empty(K, dtype=torch.float64, device="cuda")
    ctx.ode_eval_tensors(native.MIOC_ODE_FISHING, du, obj.T0, obj.T1, Jnew, None)
    dec = torch.empty(K, dtype=torch.int32, device="cuda")
    ctx.trm_decide_tensors(Jold, Jnew, outs[1], outs[2], outs[3], par.sigma, dec)
    ctx.synchronize()
    dfd, ud = df.cpu().numpy(), du.cpu().numpy()
    for k in range(4):
        host = native.Context(0)
        host.set_levels(lt)
        host.set_cost(par.p, par.beta)
        host.bellman(dfd[k].T, xs[k], B, obj.tau)  # the device gradient, so the DP inputs are identical
        u, _, _ = host.backtrack(B)
        assert np.array_equal(u, ud[k].T), k
        iv, to, tn, pr = host.pred()
        assert pr == outs[3][k].item() and tn == outs[2][k].item(), k
        obj.x[:, :] = u
        jn = mioc.eval_f_(obj)
        assert abs(jn - Jnew[k].item()) <= 1e-12 * abs(jn), k
        host.close()
    assert set(np.unique(dec.cpu().numpy())) <= {0, 1, 2}
    ctx.close()
