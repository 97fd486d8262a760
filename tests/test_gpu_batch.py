"""GPU parity of the batch path (BASELINE config C5: 1024 random-start bellman_TRM! subproblems).

The restarts mirror multi-trust.jl:53 (`x0 = rand_func(obj)`, HelpFunctions.jl:204-225): every subproblem
has its own df and a rand_func_int-shaped u_old.  The batch runs through mioc_bellman_batch_device /
mioc_backtrack_batch_device, one workgroup per subproblem (the fused small-state DP), and is checked
  * restart by restart against an independent device algorithm (the per-step generic sweep) for all 1024,
  * against the CPU oracle (HelpFunctions.jl:20-124) at the full nt = 4096 for a seeded subset of restarts:
    u, Φ* and the argmin table U on sampled steps (every cell the reference writes).
"""
import numpy as np
import pytest

from mioc import native
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_INF, P_ONE, Levels

pytestmark = pytest.mark.gpu


def _batch(cfg, K, nt=None, k0=0):
    import torch
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(k0, k0 + K):
        _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=lt)
        dfs.append(df)
        uos.append(uo)
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
    return lt, dfs, uos, ddf, duo


def _run(lt, cfg, algo, ddf, duo, B, Bp, opts=None):
    import torch
    K = ddf.shape[0]
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.set_option(native.MIOC_OPT_ALGO, algo)
    for o, v in (opts or {}).items():
        ctx.set_option(o, v)
    du = torch.empty_like(ddf)
    dphi = torch.empty(K, dtype=torch.float64, device="cuda")
    dst = torch.empty(K, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.bellman_batch_tensors(ddf, duo, B, cfg.dt)
    ctx.backtrack_batch_tensors(Bp, du, dphi, dst)
    ctx.synchronize()
    if algo != native.MIOC_ALGO_AUTO:
        assert ctx.last_algo() == algo
    return ctx, du.cpu().numpy(), dphi.cpu().numpy(), dst.cpu().numpy()


def test_c5_batch_1024_fused_equals_generic():
    """All 1024 C5 restarts at full size: the fused batch (AUTO must choose it) and the per-step generic
    sweep agree on every control and Φ*, at the full budget and at the halved one (multi-trust.jl:108-110)."""
    cfg = CONFIGS["C5"]
    lt, _, _, ddf, duo = _batch(cfg, 1024)
    B = cfg.B
    res = {}
    for algo in (native.MIOC_ALGO_AUTO, native.MIOC_ALGO_FUSED, native.MIOC_ALGO_GENERIC):
        ctx, u, phi, st = _run(lt, cfg, algo, ddf, duo, B, B)
        if algo == native.MIOC_ALGO_AUTO:
            assert ctx.last_algo() == native.MIOC_ALGO_FUSED_SEPARABLE
        assert np.all(st == 0)
        import torch
        du = torch.empty_like(ddf)
        dphi = torch.empty(ddf.shape[0], dtype=torch.float64, device="cuda")
        ctx.backtrack_batch_tensors(B // 2, du, dphi, None)
        ctx.synchronize()
        res[algo] = (u, phi, du.cpu().numpy(), dphi.cpu().numpy())
        ctx.close()
    g = res[native.MIOC_ALGO_GENERIC]
    for algo in (native.MIOC_ALGO_AUTO, native.MIOC_ALGO_FUSED):
        for x, y in zip(res[algo], g):
            bad = np.flatnonzero([not np.array_equal(p, q) for p, q in zip(x, y)])
            assert bad.size == 0, f"algo {algo}: restarts {bad[:8]} differ"


@pytest.mark.parametrize("algo", ["fused", "fused_separable"])
@pytest.mark.parametrize("k0", [0, 517])
def test_c5_batch_restarts_vs_oracle(oracle_c, k0, algo):
    """Seeded restarts of a 1024-batch at full nt = 4096, B = 256 against the CPU oracle: u and Φ* at B and
    B/2, and every U cell the reference writes on 64 sampled steps."""
    cfg = CONFIGS["C5"]
    K = 1024
    lt, dfs, uos, ddf, duo = _batch(cfg, K)
    algo = {"fused": native.MIOC_ALGO_FUSED, "fused_separable": native.MIOC_ALGO_FUSED_SEPARABLE}[algo]
    ctx, u, phi, st = _run(lt, cfg, algo, ddf, duo, cfg.B, cfg.B)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    rng = np.random.default_rng(k0)
    picks = sorted({k0 + int(x) for x in rng.integers(0, 512, size=4)} | {k0})
    nt = cfg.nt
    steps = sorted({0, nt - 2} | {int(x) for x in rng.integers(0, nt - 1, size=62)})
    for k in picks:
        ophi, oU = oracle_c.bellman(lv, dfs[k], uos[k], cfg.B, P_ONE, cfg.beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, cfg.B, cfg.B)
        assert np.array_equal(u[k].T, ou), f"restart {k}"
        assert phi[k] == ops and st[k] == 0, f"restart {k}: {phi[k]!r} vs {ops!r}"
        for i in steps:
            d, o = ctx.argmin_table(i, k=k), oU[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"restart {k} step {i}"
        ou2, ops2 = oracle_c.backtrack(lv, uos[k], ophi, oU, cfg.B, cfg.B // 2)
        u2, p2, _ = _halved(ctx, ddf, cfg.B // 2)
        assert np.array_equal(u2[k].T, ou2) and p2[k] == ops2, f"restart {k} at B/2"
    ctx.close()


def _halved(ctx, ddf, Bp):
    import torch
    du = torch.empty_like(ddf)
    dphi = torch.empty(ddf.shape[0], dtype=torch.float64, device="cuda")
    dst = torch.empty(ddf.shape[0], dtype=torch.int32, device="cuda")
    ctx.backtrack_batch_tensors(Bp, du, dphi, dst)
    ctx.synchronize()
    return du.cpu().numpy(), dphi.cpu().numpy(), dst.cpu().numpy()


@pytest.mark.parametrize("algo", ["fused", "fused_separable"])
@pytest.mark.parametrize("mode", ["zero", "integer", "outside", "steep"])
def test_fused_tie_heavy_and_off_grid_vs_oracle(oracle_c, mode, algo):
    """Batches whose DP is dominated by exact ties (zero / integer gradients) or whose u_old leaves the level
    grid (integral, not admissible): the fused DP against the oracle, restart by restart, every U cell."""
    cfg = CONFIGS["C5"]
    K, nt, B = 5, 80, 40
    rng = np.random.default_rng({"zero": 1, "integer": 2, "outside": 3, "steep": 4}[mode])
    beta = 1e-13 if mode == "steep" else cfg.beta  # value spread ~1e13 beta: rows leave the transform's binade
    lt = cfg.levels()
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    dfs, uos = [], []
    for k in range(K):
        _, df, uo = make_inputs(cfg, k=100 + k, nt=nt, levels=lt)
        if mode == "zero":
            df = np.zeros_like(df)
        elif mode == "integer":
            df = rng.integers(-3, 4, size=df.shape).astype(float)
        elif mode == "steep":
            df = df * 1e3
        else:
            uo = uo.copy()
            for i in rng.choice(nt, size=10, replace=False):
                uo[rng.integers(2), i] = float(rng.choice([-2, 7]))
        dfs.append(df)
        uos.append(uo)
    import torch
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
    algo = {"fused": native.MIOC_ALGO_FUSED, "fused_separable": native.MIOC_ALGO_FUSED_SEPARABLE}[algo]
    import dataclasses
    ctx, u, phi, st = _run(lt, dataclasses.replace(cfg, beta=beta), algo, ddf, duo, B, B)
    diag = ctx.diagnostics()
    if algo == native.MIOC_ALGO_FUSED_SEPARABLE:
        if mode in ("zero", "integer"):
            assert diag[0] > 0, diag  # targets with a near-tie winner went to the exact scan
        if mode == "steep":
            assert diag[1] > 0, diag  # rows outside the binade went to the exact scan
    for k in range(K):
        ophi, oU = oracle_c.bellman(lv, dfs[k], uos[k], B, P_ONE, beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, B, B)
        assert np.array_equal(u[k].T, ou) and phi[k] == ops, f"{mode} restart {k}"
        for i in range(nt - 1):
            d, o = ctx.argmin_table(i, k=k), oU[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"{mode} restart {k} step {i}"
    ctx.close()


@pytest.mark.parametrize("key,K", [("C2", 1024), ("C3", 256)])
def test_pinf_batch_vs_generic_and_oracle(oracle_c, key, K):
    """p = Inf restarts on the C2 / C3 shapes (multi-trust.jl:183-189 runs them at p = Inf): the class collapse
    batch (per-thread class tables, banded walk) against the generic sweep for every restart, at B and B/2, and
    against the oracle at full nt for a seeded subset; a zero-gradient batch makes every step a tie."""
    import torch
    cfg = CONFIGS[key]
    lt, dfs, uos, ddf, duo = _batch(cfg, K)
    res = {}
    for algo in (native.MIOC_ALGO_PINF, native.MIOC_ALGO_GENERIC):
        ctx, u, phi, st = _run(lt, cfg, algo, ddf, duo, cfg.B, cfg.B)
        assert np.all(st == 0)
        u2, p2, _ = _halved(ctx, ddf, cfg.B // 2)
        res[algo] = (u, phi, u2, p2)
        ctx.close()
    for x, y in zip(res[native.MIOC_ALGO_PINF], res[native.MIOC_ALGO_GENERIC]):
        bad = np.flatnonzero([not np.array_equal(p, q) for p, q in zip(x, y)])
        assert bad.size == 0, f"restarts {bad[:8]} differ"
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    u, phi = res[native.MIOC_ALGO_PINF][:2]
    rng = np.random.default_rng(K)
    for k in sorted({0, K - 1} | {int(x) for x in rng.integers(0, K, size=2)}):
        ophi, oU = oracle_c.bellman(lv, dfs[k], uos[k], cfg.B, P_INF, cfg.beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, cfg.B, cfg.B)
        assert np.array_equal(u[k].T, ou) and phi[k] == ops, f"restart {k}"
    # zero gradient: every level of a class has the same K, so every step is a tie that the first rank must win
    z = torch.zeros_like(ddf[:8])
    ctx, u, phi, st = _run(lt, cfg, native.MIOC_ALGO_PINF, z, duo[:8].contiguous(), cfg.B, cfg.B)
    assert ctx.diagnostics()[3] == 0
    for k in range(8):
        ophi, oU = oracle_c.bellman(lv, np.zeros_like(dfs[k]), uos[k], cfg.B, P_INF, cfg.beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, cfg.B, cfg.B)
        assert np.array_equal(u[k].T, ou) and phi[k] == ops, f"zero-gradient restart {k}"
    ctx.close()


@pytest.mark.parametrize("nt", [3, 17, 18, 33, 34, 35, 200])
def test_pinf_banded_walk_chunk_edges_vs_oracle(oracle_c, nt):
    """The banded p = Inf walk (a band of each R row staged in LDS) at chunk-boundary step counts, against the
    oracle restart by restart: C2 levels (B = 819, so the band is narrower than a row) and a budget small enough
    (B = 5) that the whole row is staged."""
    cfg = CONFIGS["C2"]
    lt, dfs, uos, ddf, duo = _batch(cfg, 6, nt=nt)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    for B in (cfg.B, 5):
        ctx, u, phi, st = _run(lt, cfg, native.MIOC_ALGO_PINF, ddf, duo, B, B)
        for k in range(6):
            ophi, oU = oracle_c.bellman(lv, dfs[k], uos[k], B, P_INF, cfg.beta, cfg.dt)
            ou, ops = oracle_c.backtrack(lv, uos[k], ophi, oU, B, B)
            assert np.array_equal(u[k].T, ou) and phi[k] == ops and st[k] == 0, f"nt={nt} B={B} restart {k}"
        ctx.close()


def test_batch_multi_contexts_equal_single_batch():
    """mioc_batch_multi (SURVEY §8 b): a C5 batch split over two contexts on the one visible device (each block
    from its own host thread) equals the single-context device batch restart by restart, at B and B/2."""
    cfg = CONFIGS["C5"]
    K = 96
    lt, dfs, uos, ddf, duo = _batch(cfg, K, nt=512)
    ctxs = []
    for _ in range(2):
        c = native.Context(0)
        c.set_levels(lt)
        c.set_cost(cfg.p, cfg.beta)
        ctxs.append(c)
    hdf, huo = ddf.cpu().numpy(), duo.cpu().numpy()
    for Bu in (cfg.B, cfg.B // 2):
        u, phi, st = native.batch_multi(ctxs, hdf, huo, cfg.B, cfg.dt, Bu)
        ref, ru, rphi, rst = _run(lt, cfg, native.MIOC_ALGO_AUTO, ddf, duo, cfg.B, Bu)
        assert np.array_equal(u, ru) and np.array_equal(phi, rphi) and np.array_equal(st, rst)
        ref.close()
    with pytest.raises(native.MiocNativeError):
        native.batch_multi([ctxs[0], ctxs[0]], hdf, huo, cfg.B, cfg.dt)
    for c in ctxs:
        c.close()
