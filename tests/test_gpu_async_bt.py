"""GPU: the p = Inf backtrack on the context's second stream, overlapping the next DP (two DP slots of inputs and
p = Inf tables, mioc_api.cpp run_backtrack / begin_dp / join_bt).

Interleaved sequences on ONE context -- bellman(A), backtrack(A), bellman(B), backtrack(B), ... with no host sync in
between, the halving path (several backtracks of one DP at different budgets), a p = 1 separable DP in between (its
backtrack runs on the first stream and must wait for the p = Inf one still in flight), the host-array entry points --
must give bit for bit what a fresh context gives for each problem alone, synchronised after every call.  Problems are
the reference's doubletank shape (C2, SOS1, p = Inf, multi-trust.jl:183-189): K = 1 (segmented walk) and K = 96
(one serial walk per subproblem), plus an 8^3 separable case.
"""
import numpy as np
import pytest

from mioc import native
from mioc.synth import CONFIGS, make_inputs

pytestmark = pytest.mark.gpu


def _problem(cfg, K, k0, nt):
    import torch
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(k0, k0 + K):
        _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=lt)
        dfs.append(df.T)
        uos.append(uo.T)
    ddf = torch.tensor(np.ascontiguousarray(np.stack(dfs)), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack(uos)), dtype=torch.float64, device="cuda")
    return lt, ddf, duo


def _ctx(lt, cfg):
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    return ctx


def _alone(lt, cfg, ddf, duo, budgets):
    """Each budget's (u, Φ*, status) on a fresh context, synchronised after every call."""
    import torch
    K = ddf.shape[0]
    out = []
    with _ctx(lt, cfg) as ctx:
        ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
        ctx.synchronize()
        for Bp in budgets:
            du = torch.empty_like(ddf)
            dphi = torch.empty(K, dtype=torch.float64, device="cuda")
            dst = torch.empty(K, dtype=torch.int32, device="cuda")
            ctx.backtrack_batch_tensors(Bp, du, dphi, dst)
            ctx.synchronize()
            out.append((du.cpu().numpy(), dphi.cpu().numpy(), dst.cpu().numpy()))
    return out


@pytest.mark.parametrize("K", [1, 96])
def test_interleaved_pinf_dps_equal_alone(K):
    import torch
    cfg = CONFIGS["C2"]
    nt = 1024
    probs = [_problem(cfg, K, 1000 * q, nt) for q in range(4)]
    budgets = [(cfg.B,), (cfg.B, cfg.B // 2, cfg.B // 5), (cfg.B,), (cfg.B // 3,)]
    lt = probs[0][0]
    got = []
    with _ctx(lt, cfg) as ctx:
        ctx.set_option(native.MIOC_OPT_TIMING, 1)
        for (lt_, ddf, duo), bs in zip(probs, budgets):
            ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
            outs = []
            for Bp in bs:  # the halving path: several backtracks of one DP, no sync in between
                du = torch.empty_like(ddf)
                dphi = torch.empty(K, dtype=torch.float64, device="cuda")
                dst = torch.empty(K, dtype=torch.int32, device="cuda")
                ctx.backtrack_batch_tensors(Bp, du, dphi, dst)
                outs.append((du, dphi, dst))
            got.append(outs)
        ctx.synchronize()
        assert ctx.last_algo() == native.MIOC_ALGO_PINF
        assert ctx.diagnostics()[6] == 0
        got = [[(a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy()) for a, b, c in outs] for outs in got]
    for q, ((lt_, ddf, duo), bs) in enumerate(zip(probs, budgets)):
        ref = _alone(lt_, cfg, ddf, duo, bs)
        for r, (g, e) in enumerate(zip(got[q], ref)):
            assert np.array_equal(g[2], e[2]), f"problem {q} budget {bs[r]}: status"
            assert np.array_equal(g[0], e[0]), f"problem {q} budget {bs[r]}: u"
            assert np.array_equal(g[1], e[1]), f"problem {q} budget {bs[r]}: phi*"


def test_pinf_then_separable_then_pinf_and_ranks():
    """A p = Inf backtrack in flight, then a p = 1 separable DP and backtrack on the same context (the latter on the
    first stream, after the former), then p = Inf again; ranks read back through mioc_get_ranks_device."""
    import torch
    cfg = CONFIGS["C2"]
    nt = 600
    ltA, dfA, uoA = _problem(cfg, 8, 7, nt)
    ltC, dfC, uoC = _problem(cfg, 8, 77, nt)
    # an 8^3 grid of consecutive levels at p = 1: the separable transform (k_sdt_run<3>)
    from mioc.iterators import LevelTable
    lv3 = LevelTable([list(range(8))] * 3)  # the product iterator
    rng = np.random.default_rng(5)
    df3 = rng.standard_normal((1, 40, 3))
    uo3 = rng.integers(0, 8, size=(1, 40, 3)).astype(float)
    d_df3 = torch.tensor(df3, dtype=torch.float64, device="cuda")
    d_uo3 = torch.tensor(uo3, dtype=torch.float64, device="cuda")

    def run(ctx, lt, p, beta, ddf, duo, B, dt):
        ctx.set_levels(lt)
        ctx.set_cost(p, beta)
        K = ddf.shape[0]
        du = torch.empty_like(ddf)
        dphi = torch.empty(K, dtype=torch.float64, device="cuda")
        dst = torch.empty(K, dtype=torch.int32, device="cuda")
        rk = torch.empty((K, ddf.shape[1]), dtype=torch.int32, device="cuda")
        ctx.bellman_batch_tensors(ddf, duo, B, dt)
        ctx.backtrack_batch_tensors(B, du, dphi, dst)
        ctx.ranks_tensor(rk)
        return du, dphi, dst, rk

    seq = [(ltA, cfg.p, cfg.beta, dfA, uoA, cfg.B, cfg.dt), (lv3, 1.0, 0.3, d_df3, d_uo3, 20, 0.5),
           (ltC, cfg.p, cfg.beta, dfC, uoC, cfg.B, cfg.dt)]
    with native.Context(0) as ctx:
        got = [run(ctx, *a) for a in seq]
        ctx.synchronize()
        got = [[t.cpu().numpy() for t in g] for g in got]
    for q, a in enumerate(seq):
        with native.Context(0) as ctx:
            e = run(ctx, *a)
            ctx.synchronize()
            e = [t.cpu().numpy() for t in e]
        for name, x, y in zip(("u", "phi*", "status", "ranks"), got[q], e):
            assert np.array_equal(x, y), f"step {q}: {name}"


def test_host_entry_points_after_async_backtrack():
    """The host-array backtrack (mioc_backtrack) and pred read a p = Inf backtrack's results on the first stream."""
    cfg = CONFIGS["C2"]
    lt, df, uo = make_inputs(cfg, k=3, nt=800)
    with _ctx(lt, cfg) as a, _ctx(lt, cfg) as b:
        a.bellman(df, uo, cfg.B, cfg.dt)
        u1, p1, _ = a.backtrack(cfg.B)
        u2, p2, _ = a.backtrack(cfg.B // 2)
        pa = a.pred()
        b.bellman(df, uo, cfg.B, cfg.dt)
        b.synchronize()
        v2, q2, _ = b.backtrack(cfg.B // 2)
        b.synchronize()
        pb = b.pred()
        v1, q1, _ = b.backtrack(cfg.B)
        assert np.array_equal(u1, v1) and p1 == q1
        assert np.array_equal(u2, v2) and p2 == q2
        # pred of each context's last backtrack: a's is B // 2, b's pred was taken after its B // 2 backtrack too
        assert pa == pb
