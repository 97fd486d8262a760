"""GPU parity of the round-3 fused separable DP (mioc_fsep.hip: two lanes per row, the front updated in place,
optionally S row segments per subproblem chained by an outbox ring) against the CPU oracle (HelpFunctions.jl:20-124)
and against the one-lane-per-row kernel of mioc_fused.hip, every U cell the reference writes."""
import dataclasses

import numpy as np
import pytest

from mioc import native
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_ONE, Levels

pytestmark = pytest.mark.gpu


def _tensors(dfs, uos):
    import torch
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
    return ddf, duo


def _solve(lt, cfg, ddf, duo, B, seg, Bp=None, spin=None):
    import torch
    K = ddf.shape[0]
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_FUSED_SEPARABLE)
    ctx.set_option(native.MIOC_OPT_FSEP_SEGMENTS, seg)
    if spin is not None:
        ctx.set_option(native.MIOC_OPT_SPIN_LIMIT, spin)
    du = torch.empty_like(ddf)
    dphi = torch.empty(K, dtype=torch.float64, device="cuda")
    dst = torch.empty(K, dtype=torch.int32, device="cuda")
    ctx.bellman_batch_tensors(ddf, duo, B, cfg.dt)
    ctx.backtrack_batch_tensors(B if Bp is None else Bp, du, dphi, dst)
    ctx.synchronize()
    return ctx, du.cpu().numpy(), dphi.cpu().numpy(), dst.cpu().numpy()


def _inputs(cfg, mode, K, nt, seed):
    rng = np.random.default_rng(seed)
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(K):
        _, df, uo = make_inputs(cfg, k=300 + k, nt=nt, levels=lt)
        if mode == "zero":
            df = np.zeros_like(df)
        elif mode == "integer":
            df = rng.integers(-3, 4, size=df.shape).astype(float)
        elif mode == "steep":
            df = df * 1e3
        elif mode == "outside":
            uo = uo.copy()
            for i in rng.choice(nt, size=8, replace=False):
                uo[rng.integers(2), i] = float(rng.choice([-2, 7]))
        dfs.append(df)
        uos.append(uo)
    return lt, dfs, uos


@pytest.mark.parametrize("seg", [-1, 1, 2, 4])
@pytest.mark.parametrize("mode", ["gauss", "zero", "integer", "outside", "steep"])
def test_fsep_segments_vs_oracle(oracle_c, mode, seg):
    """C5 levels (6x6), B = 200 (segments of 128 / 64 rows plus a short last one), nt = 40: u, Φ* at B and B/2
    and every U cell against the oracle, for the old kernel (-1), one workgroup per subproblem (1) and 2 / 4 row
    segments; tie-heavy, off-grid and out-of-binade inputs exercise the exact scans."""
    cfg = CONFIGS["C5"]
    K, nt, B = 3, 40, 200
    lt, dfs, uos = _inputs(cfg, mode, K, nt, {"gauss": 0, "zero": 1, "integer": 2, "outside": 3, "steep": 4}[mode])
    beta = 1e-13 if mode == "steep" else cfg.beta
    cfgb = dataclasses.replace(cfg, beta=beta)
    ddf, duo = _tensors(dfs, uos)
    ctx, u, phi, st = _solve(lt, cfgb, ddf, duo, B, seg)
    diag = ctx.diagnostics()
    # an off-grid u_old reaches further than a segment's outbox rows: such a DP runs unsegmented
    want = 0 if seg < 0 else (1 if mode == "outside" else seg)
    assert diag[8] == want and diag[3] == 0 and diag[6] == 0, diag
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    for k in range(K):
        ophi, oU = oracle_c.bellman(lv, dfs[k], uos[k], B, P_ONE, beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, B, B)
        assert np.array_equal(u[k].T, ou) and phi[k] == ops, f"{mode} restart {k}"
        for i in range(nt - 1):
            d, o = ctx.argmin_table(i, k=k), oU[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"{mode} restart {k} step {i}"
    ctx.close()


def test_fsep_c5_full_size_segments_equal():
    """C5 at full size (nt = 4096, B = 256) with a batch too small to fill the GPU: the automatic choice splits
    every subproblem into row segments (diagnostics [8] > 1); controls, Φ* and sampled U tables equal those of
    one workgroup per subproblem and of the one-lane-per-row kernel, at B and B/2."""
    cfg = CONFIGS["C5"]
    K = 16
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(K):
        _, df, uo = make_inputs(cfg, k=k, levels=lt)
        dfs.append(df)
        uos.append(uo)
    ddf, duo = _tensors(dfs, uos)
    res = {}
    steps = [0, 1, 777, 2048, cfg.nt - 2]
    for seg in (0, 1, -1):
        ctx, u, phi, st = _solve(lt, cfg, ddf, duo, cfg.B, seg)
        assert np.all(st == 0)
        diag = ctx.diagnostics()
        if seg == 0:
            assert diag[8] > 1, diag
        tabs = [ctx.argmin_table(i, k=k) for k in (0, K - 1) for i in steps]
        ctx2, u2, phi2, _ = _solve(lt, cfg, ddf, duo, cfg.B, seg, Bp=cfg.B // 2)
        res[seg] = (u, phi, u2, phi2, tabs)
        ctx.close()
        ctx2.close()
    for seg in (0, 1):
        for x, y in zip(res[seg][:4], res[-1][:4]):
            assert np.array_equal(x, y), f"segments {seg}"
        for a, b in zip(res[seg][4], res[-1][4]):
            assert np.array_equal(a, b), f"segments {seg}: U table"


def test_fsep_segment_wait_timeout_redoes_dp():
    """A segmented launch whose hand-off waits give up at once (spin limit 1) is abandoned and the DP redone
    with one workgroup per subproblem (diagnostics [6] counts it); the results equal a normal run."""
    cfg = CONFIGS["C5"]
    lt, dfs, uos = _inputs(cfg, "gauss", 4, 300, 7)
    ddf, duo = _tensors(dfs, uos)
    ctx, u, phi, st = _solve(lt, cfg, ddf, duo, cfg.B, 2, spin=1)
    diag = ctx.diagnostics()
    assert diag[6] >= 1 and diag[3] == 0, diag
    ref, ru, rphi, rst = _solve(lt, cfg, ddf, duo, cfg.B, 1)
    assert np.array_equal(u, ru) and np.array_equal(phi, rphi) and np.array_equal(st, rst)
    ctx.close()
    ref.close()
