"""GPU parity of the trust-region quantities around the DP: mioc_pred, mioc_pred_batch_device,
mioc_tv_device and mioc_trm_decide_device against the oracle's restatement of multi-trust.jl:117-158 and TV_p
(HelpFunctions.jl:251-268).

Bars: TV_p bit-exact (p = 1, Inf, integer p via the host table, MIOC_P_TABLE); int_val and pred bit-exact against
the restatement in the same loop order (plain products, and fma with MIOC_OPT_PRED_FMA = 1), and the two within
1e-12 of the scale Δt·Σ|∇f|·|u_old − u| (the reference's BLAS ddot may use either).
"""
import dataclasses
import math

import numpy as np
import pytest

from mioc import native
from mioc.iterators import LevelTable, product_iterator
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import (P_INF, P_INTLUT, P_ONE, P_TABLE, Levels, pred_py, trm_decide_py, tv_p_kind,
                           tv_p_py)

pytestmark = pytest.mark.gpu


def _kind(ctx_tab, p, levels):
    pk, pint, tab = native.cost_spec(p, levels=levels)
    return pk, pint, tab


def _olv(lt):
    return Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])


def _tv_dev(ctx, u_list):
    import torch
    du = torch.tensor(np.ascontiguousarray(np.stack([u.T for u in u_list])), dtype=torch.float64, device="cuda")
    out = torch.empty(len(u_list), dtype=torch.float64, device="cuda")
    ctx.tv_tensors(du, out)
    ctx.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("p", [1, math.inf, 2, 1.5])
def test_tv_docstring_kat_and_random(p):
    """TV_p docstring vectors (HelpFunctions.jl:235-249: 8, 5.741657386773941, 5) and random integral controls."""
    nu = [[-1, 0, 1, 2, 3]] * 3
    lt = LevelTable(nu, product_iterator(nu))
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(p, 1e-3)
    pk, pint, tab = _kind(ctx, p, lt)
    u = np.array([[1, -1, 1], [3, 3, 0], [2, 2, 1]], dtype=float)
    rng = np.random.default_rng(11)
    us = [u] + [rng.integers(-1, 4, size=(3, n)).astype(float) for n in (1, 2, 64, 1000, 5000)]
    got = _tv_dev(ctx, us[:1])
    want = {1: 8.0, math.inf: 5.0, 2: 5.741657386773941}.get(p)
    if want is not None:
        assert got[0] == want
    for x in us:
        d = _tv_dev(ctx, [x])[0]
        assert d == tv_p_kind(x, pk, pint, tab, _olv(lt)), (p, x.shape)
        assert abs(d - tv_p_py(x, p)) <= 1e-12 * max(1.0, d)
    # a batch of different controls at once
    xs = [rng.integers(-1, 4, size=(3, 777)).astype(float) for _ in range(9)]
    d = _tv_dev(ctx, xs)
    assert [float(v) for v in d] == [tv_p_kind(x, pk, pint, tab, _olv(lt)) for x in xs]
    ctx.close()


def _scale(df, uo, u, dt):
    return dt * float(np.sum(np.abs(df) * np.abs(uo - u))) + 1e-300


@pytest.mark.parametrize("cfg_name,nt", [("C1", None), ("C2", None), ("C5", None), ("C4", 4096), ("C4", None)])
def test_pred_single_vs_oracle(cfg_name, nt):
    """mioc_pred after mioc_bellman/mioc_backtrack at the BASELINE configs (C4 at its full nt = 65536 too), at
    the full budget and after the halving path's re-backtrack (multi-trust.jl:108-110)."""
    cfg = CONFIGS[cfg_name]
    lt, df, uo = make_inputs(cfg, nt=nt)
    pk, pint, tab = native.cost_spec(cfg.p, levels=lt)
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    for Bu in (cfg.B, cfg.B // 2):
        u, _, _ = ctx.backtrack(Bu)
        ctx.set_option(native.MIOC_OPT_PRED_FMA, 0)
        iv, to, tn, pr = ctx.pred()
        ctx.set_option(native.MIOC_OPT_PRED_FMA, 1)
        ivf, to2, tn2, prf = ctx.pred()
        eto = tv_p_kind(uo, pk, pint, tab, _olv(lt))
        etn = tv_p_kind(u, pk, pint, tab, _olv(lt))
        assert to == eto and tn == etn and to2 == eto and tn2 == etn
        eiv, epr = pred_py(df, uo, u, cfg.dt, cfg.beta, eto, etn)
        assert iv == eiv and pr == epr, (iv, eiv)
        eivf, eprf = pred_py(df, uo, u, cfg.dt, cfg.beta, eto, etn, fma=True)
        assert ivf == eivf and prf == eprf
        assert abs(iv - ivf) <= 1e-12 * _scale(df, uo, u, cfg.dt)
    ctx.close()


def test_pred_batch_c5_vs_oracle():
    """mioc_pred_batch_device for the 1024-restart C5 batch: TV exact for every restart, int_val / pred bit-exact
    for a seeded subset; the decision kernel on the resulting pred with synthetic J values."""
    import torch
    cfg = CONFIGS["C5"]
    K = 1024
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(K):
        _, df, uo = make_inputs(cfg, k=k, levels=lt)
        dfs.append(df)
        uos.append(uo)
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    du = torch.empty_like(ddf)
    ctx.backtrack_batch_tensors(cfg.B, du)
    outs = [torch.empty(K, dtype=torch.float64, device="cuda") for _ in range(4)]
    ctx.pred_batch_tensors(*outs)
    ctx.synchronize()
    iv, to, tn, pr = [o.cpu().numpy() for o in outs]
    u = du.cpu().numpy()
    # p = 1: TV terms are integers, so any summation order is exact -- vectorised expected values
    assert np.array_equal(to, np.abs(np.diff(np.stack(uos), axis=2)).sum(axis=(1, 2)))
    assert np.array_equal(tn, np.abs(np.diff(u, axis=1)).sum(axis=(1, 2)))
    rng = np.random.default_rng(3)
    for k in sorted({0, K - 1} | {int(x) for x in rng.integers(0, K, size=6)}):
        eiv, epr = pred_py(dfs[k], uos[k], u[k].T, cfg.dt, cfg.beta, float(to[k]), float(tn[k]))
        assert iv[k] == eiv and pr[k] == epr, k
    # the step decision (multi-trust.jl:127-158) on the device vs the restatement
    Jo = torch.tensor(rng.standard_normal(K), dtype=torch.float64, device="cuda")
    Jn = Jo - torch.tensor(rng.standard_normal(K) * 1e-3, dtype=torch.float64, device="cuda")
    dec = torch.empty(K, dtype=torch.int32, device="cuda")
    ared = torch.empty(K, dtype=torch.float64, device="cuda")
    ctx.trm_decide_tensors(Jo, Jn, outs[1], outs[2], outs[3], 0.5, dec, ared)
    ctx.synchronize()
    dec, ared = dec.cpu().numpy(), ared.cpu().numpy()
    Jo, Jn = Jo.cpu().numpy(), Jn.cpu().numpy()
    for k in range(K):
        ea, ed = trm_decide_py(float(Jo[k]), float(Jn[k]), float(to[k]), float(tn[k]), float(pr[k]), cfg.beta, 0.5)
        assert ared[k] == ea and dec[k] == ed, k
    ctx.close()


def test_decide_edge_cases():
    """pred <= 0 stops before the ared test; NaN pred / ared fall through to accept, as the reference's if-chain."""
    import torch
    vals = [(1.0, 0.5, 0.0, 0.0, 0.0), (1.0, 0.5, 0.0, 0.0, -0.0), (1.0, 0.99, 0.0, 0.0, 1.0),
            (1.0, 0.0, 0.0, 0.0, 1.0), (1.0, 0.0, 0.0, 0.0, float("nan")), (float("nan"), 0.0, 0.0, 0.0, 1.0),
            (2.0, 1.0, 3.0, 1.0, 1.0 + 2e-3), (2.0, 1.0, 1.0, 3.0, 1e-300)]
    cols = [torch.tensor([v[i] for v in vals], dtype=torch.float64, device="cuda") for i in range(5)]
    ctx = native.Context(0)
    nu = [[0, 1]]
    ctx.set_levels(LevelTable(nu, product_iterator(nu)))
    ctx.set_cost(1, 1e-3)
    dec = torch.empty(len(vals), dtype=torch.int32, device="cuda")
    ctx.trm_decide_tensors(*cols, 0.5, dec)
    ctx.synchronize()
    for v, d in zip(vals, dec.cpu().numpy()):
        assert d == trm_decide_py(*v, 1e-3, 0.5)[1], v
    ctx.close()


def test_pred_errors():
    """Integer p with an off-grid u_old whose jump key exceeds the host table, and pred before a backtrack."""
    cfg = dataclasses.replace(CONFIGS["C5"], p=2)
    lt, df, uo = make_inputs(cfg, nt=64)
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(2, cfg.beta)
    with pytest.raises(native.MiocNativeError):
        ctx.pred()
    uo = uo.copy()
    uo[:, 10] = [-7.0, 12.0]  # |d|^2 sums up to 19^2 + 12^2 > the table's 2 * 5^2
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    ctx.backtrack(cfg.B)
    with pytest.raises(native.MiocNativeError, match="TV_p"):
        ctx.pred()
    ctx.close()
