"""GPU parity: libmioc (through the C ABI) against the CPU oracle and the golden fixtures.

Bar: the control u (hence the switching pattern) and Φ* bit-identical to the oracle; pred within
1e-12 relative.  Full-size configs that the oracle finishes in seconds (C1, C2, C3, one C5 restart)
are compared directly; the 4096-level C4 config is compared on truncated fixtures and, at full
size, through size-independent properties (exact objective recomputation along the returned path,
exact budget, admissibility, DP(B)/backtrack(B') == DP(B')/backtrack(B'), algorithm agreement).
"""
import math

import numpy as np
import pytest

from conftest import golden_files, load_golden
from mioc import native
from mioc.iterators import LevelTable
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_INF, P_INTLUT, P_ONE, Levels

pytestmark = pytest.mark.gpu

ALGOS_PINF = (native.MIOC_ALGO_PINF, native.MIOC_ALGO_GENERIC)


def _ctx(levels, p_kind, beta, algo, p_int=1, table=None):
    ctx = native.Context(0)
    ctx.set_levels(levels)
    ctx.set_cost(None, beta, table=table, p_int=p_int, p_kind=p_kind)
    ctx.set_option(native.MIOC_OPT_ALGO, algo)
    return ctx


def _oracle_levels(lt):
    return Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])


def _algos(p_kind, lt=None, B=None):
    fused = (native.MIOC_ALGO_FUSED,) if lt is not None and B is not None and native.fused_eligible(lt.L, B) else ()
    if p_kind == P_ONE and lt is not None and B is not None and native.fused_separable_eligible(lt, B):
        fused += (native.MIOC_ALGO_FUSED_SEPARABLE,)
    if p_kind == P_INF:
        return ALGOS_PINF + fused
    if p_kind == P_ONE and lt is not None and native.separable_eligible(lt):
        return (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_PYRAMID, native.MIOC_ALGO_SEPARABLE) + fused
    if p_kind == P_ONE and lt is not None and native.pyramid_eligible(lt):
        return (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_PYRAMID) + fused
    return (native.MIOC_ALGO_GENERIC,) + fused


def _assert_U(ctx, U, n, tag):
    """Every cell of the reference's U table (HelpFunctions.jl:74) that the reference writes equals the
    device's argmin (mioc_get_argmin_table), step by step."""
    for i in range(n - 1):
        d = ctx.argmin_table(i)
        o = U[:, :, i]
        m = o >= 0
        bad = np.argwhere(m & (d != o))
        assert bad.size == 0, f"{tag} step {i}: (c, g) {bad[:5].tolist()} device {d[m & (d != o)][:5]} ref {o[m & (d != o)][:5]}"


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("/")[-1][:-4])
def test_golden_fixtures(path):
    g = load_golden(path)
    lt = LevelTable(g["nu"], g["tuple_list"])
    table = g["wtab"] if g["wtab"].size else None
    for algo in _algos(g["p_kind"], lt, g["B"]):
        ctx = _ctx(lt, g["p_kind"], g["beta"], algo, p_int=g["p_int"], table=table)
        ctx.bellman(g["df"], g["u_old"], g["B"], g["dt"])
        assert ctx.last_algo() == algo
        u, phi, sw = ctx.backtrack(g["Bp"])
        assert np.array_equal(u, g["u"]), f"{g['name']} algo={algo}"
        assert phi == g["phi_star"][0], f"{g['name']} algo={algo}: {phi!r} vs {g['phi_star'][0]!r}"
        assert np.array_equal(sw[1:], np.any(g["u"][:, 1:] != g["u"][:, :-1], axis=0))
        ctx.close()


def _random_case(seed):
    rng = np.random.default_rng(1000 + seed)
    shapes = [([[0, 1]] * 3, "sos1"), ([[0, 1, 2], [0, 1]], "prod"), ([[-2, 0, 3]], "prod"),
              ([list(range(4))] * 2, "prod"), ([[0, 1]] * 4, "prod"), ([list(range(6))] * 2, "prod"),
              ([list(range(8)), list(range(-1, 3))], "prod"), ([list(range(4))] * 3, "prod"),
              ([list(range(8))] * 2, "prod")]
    nu, kind = shapes[seed % len(shapes)]
    lv = Levels.product(nu) if kind == "prod" else Levels.bounded_sum(nu, 1, 1)
    n = int(rng.integers(1, 40))
    B = int(rng.integers(0, 30))
    mode = seed % 4
    if mode == 0:
        df = np.zeros((lv.M, n))                              # all ties
    elif mode == 1:
        df = rng.integers(-4, 5, size=(lv.M, n)).astype(float)  # integer gradients: many exact ties
    else:
        df = rng.standard_normal((lv.M, n))
    uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(n)], dtype=np.float64).T
    return lv, df, uo, B, rng


@pytest.mark.parametrize("seed", range(72))
def test_random_vs_oracle(oracle_c, seed):
    lv, df, uo, B, rng = _random_case(seed)
    pk = [P_ONE, P_INF][seed % 2]
    beta = [1e-3, 0.25, 0.1][seed % 3]
    dt = [0.5, 1 / 3, 2.0 ** -6][seed % 3]
    phi, U = oracle_c.bellman(lv, df, uo, B, pk, beta, dt)
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    budgets = sorted({B, B // 2, 0, int(rng.integers(0, B + 1))})
    for algo in _algos(pk, lt, B):
        ctx = _ctx(lt, pk, beta, algo)
        ctx.bellman(df, uo, B, dt)
        if algo != native.MIOC_ALGO_PINF:
            _assert_U(ctx, U, df.shape[1], f"seed={seed} algo={algo}")
        for Bp in budgets:  # one DP, several budgets: the halving reuse of multi-trust.jl:108-110
            try:
                ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
            except Exception:
                with pytest.raises(native.MiocNativeError):
                    ctx.backtrack(Bp)
                continue
            u, ps, _ = ctx.backtrack(Bp)
            assert np.array_equal(u, ou), f"seed={seed} algo={algo} Bp={Bp}"
            assert ps == ops, f"seed={seed} algo={algo} Bp={Bp}: {ps!r} vs {ops!r}"
        ctx.close()


def test_p2_lut_and_table_kinds_vs_oracle(oracle_c):
    cfg = CONFIGS["C5"]
    lt, df, uo = make_inputs(cfg, nt=40)
    lv = _oracle_levels(lt)
    B = 20
    k, pint, tab = native.cost_spec(2, levels=lt)
    phi, U = oracle_c.bellman(lv, df, uo, B, P_INTLUT, 1e-3, cfg.dt, p_int=2, wtab=tab)
    ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, B)
    nv = lt.nuval
    S = (np.abs(nv[:, None, :] - nv[None, :, :]) ** 2).sum(axis=2).astype(int)
    for algo in (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_FUSED):
        ctx = _ctx(lt, k, 1e-3, algo, p_int=pint, table=tab)
        ctx.bellman(df, uo, B, cfg.dt)
        u, ps, _ = ctx.backtrack(B)
        assert np.array_equal(u, ou) and ps == ops, f"algo={algo}"
        _assert_U(ctx, U, df.shape[1], f"p2 lut algo={algo}")
        # the same weights as a full pair table (MIOC_P_TABLE) must give the same answer
        ctx2 = _ctx(lt, native.MIOC_P_TABLE, 1e-3, algo, table=tab[S].reshape(-1))
        ctx2.bellman(df, uo, B, cfg.dt)
        u2, ps2, _ = ctx2.backtrack(B)
        assert np.array_equal(u2, ou) and ps2 == ops, f"algo={algo}"


@pytest.mark.parametrize("key", ["C1", "C2", "C3"])
def test_full_size_sos1_configs_vs_oracle(oracle_c, key):
    """C1/C2/C3 at their full BASELINE sizes (3-of-8 SOS1 levels, p=Inf): both algorithms."""
    cfg = CONFIGS[key]
    lt, df, uo = make_inputs(cfg)
    lv = _oracle_levels(lt)
    phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_INF, cfg.beta, cfg.dt)
    for Bp in (cfg.B, cfg.B // 2, cfg.B // 8):
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, Bp)
        for algo in ALGOS_PINF + (native.MIOC_ALGO_FUSED,):
            ctx = _ctx(lt, P_INF, cfg.beta, algo)
            ctx.bellman(df, uo, cfg.B, cfg.dt)
            u, ps, _ = ctx.backtrack(Bp)
            assert np.array_equal(u, ou), f"{key} algo={algo} Bp={Bp}"
            assert ps == ops
            ctx.close()


def test_full_size_c5_restart_vs_oracle(oracle_c):
    cfg = CONFIGS["C5"]
    lt, df, uo = make_inputs(cfg, k=3)
    lv = _oracle_levels(lt)
    phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_ONE, cfg.beta, cfg.dt)
    ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, cfg.B)
    for algo in (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_FUSED, native.MIOC_ALGO_FUSED_SEPARABLE):
        ctx = _ctx(lt, P_ONE, cfg.beta, algo)
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        u, ps, _ = ctx.backtrack(cfg.B)
        assert np.array_equal(u, ou) and ps == ops, f"algo={algo}"


def test_full_size_c5_p2_restart_vs_oracle(oracle_c):
    """The reference's heat configuration uses p = 2 (multi-trust.jl:193-195, weights (Σ|Δ|²)^(1/2),
    HelpFunctions.jl:63-67): one C5-shape restart at the full nt = 4096, B = 256 with the integer-key LUT
    (MIOC_P_INTLUT; host weights from Python's pow, so parity with Julia's own ^ is unpinned -- DESIGN §4) against
    the oracle: u, Φ* and U on 64 sampled steps, generic sweep and fused DP."""
    cfg = CONFIGS["C5"]
    lt, df, uo = make_inputs(cfg, k=5)
    lv = _oracle_levels(lt)
    k, pint, tab = native.cost_spec(2, levels=lt)
    phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_INTLUT, cfg.beta, cfg.dt, p_int=2, wtab=tab)
    steps = sorted(set(np.linspace(0, cfg.nt - 2, 64).astype(int).tolist()))
    for algo in (native.MIOC_ALGO_FUSED, native.MIOC_ALGO_GENERIC):
        ctx = _ctx(lt, k, cfg.beta, algo, p_int=pint, table=tab)
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        assert ctx.last_algo() == algo
        for Bp in (cfg.B, cfg.B // 3):
            ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, Bp)
            u, ps, _ = ctx.backtrack(Bp)
            assert np.array_equal(u, ou) and ps == ops, f"algo={algo} B'={Bp}"
        for i in steps:
            d, o = ctx.argmin_table(i), U[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"algo={algo} step {i}"
        ctx.close()


def test_backtrack_budgets_device_vs_single():
    """eval_u_TRM! with one budget per subproblem (mioc_backtrack_batch_budgets_device, the halving path of
    multi-trust.jl:108-110 per restart) equals a separate backtrack at each budget; a budget outside [0, B] is
    caught on the device (no host read-back): that subproblem's status is MIOC_ESTATE and its u row NaN."""
    import torch
    cfg = CONFIGS["C5"]
    K, nt = 6, 200
    subs = [make_inputs(cfg, k=k, nt=nt)[1:] for k in range(K)]
    lt = cfg.levels()
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d, _ in subs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([u.T for _, u in subs])), dtype=torch.float64, device="cuda")
    budgets = [cfg.B, 0, 77, -1, cfg.B + 1, 5]
    for algo in (native.MIOC_ALGO_FUSED_SEPARABLE, native.MIOC_ALGO_FUSED, native.MIOC_ALGO_GENERIC):
        ctx = _ctx(lt, P_ONE, cfg.beta, algo)
        torch.cuda.synchronize()
        ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
        du = torch.empty_like(ddf)
        dphi = torch.empty(K, dtype=torch.float64, device="cuda")
        dst = torch.empty(K, dtype=torch.int32, device="cuda")
        bv = torch.tensor(budgets, dtype=torch.int32, device="cuda")
        ctx.backtrack_batch_budgets_tensors(bv, du, dphi, dst)
        ctx.synchronize()
        ub, st = du.cpu().numpy(), dst.cpu().numpy()
        for k, Bp in enumerate(budgets):
            if not 0 <= Bp <= cfg.B:
                assert st[k] == native.MIOC_ESTATE and np.all(np.isnan(ub[k])), (algo, k, Bp)
                continue
            single = _ctx(lt, P_ONE, cfg.beta, algo)
            single.bellman(*subs[k], cfg.B, cfg.dt)
            u, ps, _ = single.backtrack(Bp)
            assert st[k] == 0 and np.array_equal(ub[k].T, u) and dphi[k].item() == ps, (algo, k, Bp)
            single.close()
        ctx.close()


@pytest.mark.parametrize("algo", ["separable", "pyramid", "pinf"])
def test_backtrack_budgets_device_start_kernels(algo):
    """The per-restart budget check of the other start kernels (k_stage_argmin0 for the staging-layout DPs,
    k_pinf_start for the p=Inf collapse): a budget outside [0, B] gives that subproblem MIOC_ESTATE and a NaN u row,
    the others equal a separate backtrack at their budget (multi-trust.jl:108-110 per restart)."""
    import torch
    rng = np.random.default_rng({"separable": 31, "pyramid": 32, "pinf": 33}[algo])
    if algo == "pinf":
        cfg = CONFIGS["C2"]
        lt = cfg.levels()
        K, nt, B, beta, dt, pk = 5, 96, 40, cfg.beta, cfg.dt, P_INF
        subs = [make_inputs(cfg, k=k, nt=nt)[1:] for k in range(K)]
        aid = native.MIOC_ALGO_PINF
    else:
        lv = Levels.product([list(range(8))] * 3)
        lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
        K, nt, B, beta, dt, pk = 5, 24, 20, 1e-3, 2.0 ** -10, P_ONE
        subs = []
        for _ in range(K):
            df = rng.standard_normal((3, nt))
            uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(nt)], dtype=np.float64).T.copy()
            subs.append((df, uo))
        aid = native.MIOC_ALGO_SEPARABLE if algo == "separable" else native.MIOC_ALGO_PYRAMID
    budgets = [B, -1, B + 1, 5, 0]
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d, _ in subs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([u.T for _, u in subs])), dtype=torch.float64, device="cuda")
    ctx = _ctx(lt, pk, beta, aid)
    torch.cuda.synchronize()
    ctx.bellman_batch_tensors(ddf, duo, B, dt)
    assert ctx.last_algo() == aid
    du = torch.empty_like(ddf)
    dphi = torch.empty(K, dtype=torch.float64, device="cuda")
    dst = torch.empty(K, dtype=torch.int32, device="cuda")
    ctx.backtrack_batch_budgets_tensors(torch.tensor(budgets, dtype=torch.int32, device="cuda"), du, dphi, dst)
    ctx.synchronize()
    ub, st = du.cpu().numpy(), dst.cpu().numpy()
    for k, Bp in enumerate(budgets):
        if not 0 <= Bp <= B:
            assert st[k] == native.MIOC_ESTATE and np.all(np.isnan(ub[k])), (algo, k, Bp)
            continue
        single = _ctx(lt, pk, beta, aid)
        single.bellman(*subs[k], B, dt)
        try:
            u, ps, _ = single.backtrack(Bp)
        except native.MiocNativeError:  # no finite value within this budget: the batch row says so too
            assert st[k] != 0, (algo, k, Bp)
            single.close()
            continue
        assert st[k] == 0 and np.array_equal(ub[k].T, u) and dphi[k].item() == ps, (algo, k, Bp)
        single.close()
    ctx.close()


def _path_objective(lt, df, u, dt, beta, p_kind):
    """Φ* recomputed along a control in the reference's rounding order (HelpFunctions.jl:52-71)."""
    M, n = u.shape
    T1 = np.zeros(n)
    for m in range(M):
        T1 = T1 + (dt * df[m]) * u[m]
    if p_kind == P_INF:
        cost = np.full(n - 1, beta * 1.0)
    else:
        w = np.zeros(n - 1)
        for m in range(M):
            w = w + np.abs(u[m, 1:] - u[m, :-1])
        cost = beta * w
    K = T1[:-1] + cost
    V = T1[-1]
    for i in range(n - 2, -1, -1):
        V = K[i] + V
    return V


@pytest.mark.parametrize("p", [math.inf, 1], ids=["pinf", "p1"])
def test_full_size_c4_properties(p):
    """The 4096-level / nt=65536 / B=256 roofline config: properties that hold at any size."""
    cfg = CONFIGS["C4"]
    lt, df, uo = make_inputs(cfg)
    pk = P_INF if p == math.inf else P_ONE
    B = cfg.B
    ctx = _ctx(lt, pk, cfg.beta, native.MIOC_ALGO_AUTO)
    ctx.bellman(df, uo, B, cfg.dt)
    results = {}
    for Bp in (B, B // 2):
        u, ps, _ = ctx.backtrack(Bp)
        rows = {tuple(r) for r in lt.nuval}
        assert all(tuple(c) in rows for c in u.T)                          # admissible
        used = int(np.abs(u - uo).sum())
        assert used <= Bp                                                  # trust-region budget
        assert _path_objective(lt, df, u, cfg.dt, cfg.beta, pk) == ps      # Φ* exact along the path
        results[Bp] = (u, ps)
    # DP(B) then backtrack(B/2) == DP(B/2) then backtrack(B/2): exact-budget semantics
    ctx.bellman(df, uo, B // 2, cfg.dt)
    u2, ps2, _ = ctx.backtrack(B // 2)
    assert np.array_equal(u2, results[B // 2][0]) and ps2 == results[B // 2][1]
    if pk == P_INF:  # the collapse and the generic sweep are independent algorithms: must agree
        ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_GENERIC)
        ctx.bellman(df[:, :4096], uo[:, :4096], B, cfg.dt)
        ug, pg, _ = ctx.backtrack(B)
        ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_PINF)
        ctx.bellman(df[:, :4096], uo[:, :4096], B, cfg.dt)
        up, pp, _ = ctx.backtrack(B)
        assert np.array_equal(ug, up) and pg == pp
    ctx.close()


def test_pyramid_batch_equals_single(oracle_c):
    """K=3 subproblems through the batch API on the pyramid: per-subproblem staging, U and sphere-order
    strides.  Controls, Φ* and every written U cell equal three single runs."""
    import torch
    lt = LevelTable([list(range(8))] * 3)
    lv = _oracle_levels(lt)
    K, nt, B, beta, dt = 3, 14, 24, 1e-3, 2.0 ** -9
    rng = np.random.default_rng(42)
    dfs = [rng.standard_normal((3, nt)) for _ in range(K)]
    uos = [np.array([lt.nuval[rng.integers(lt.L)] for _ in range(nt)], dtype=np.float64).T for _ in range(K)]
    ctx = _ctx(lt, P_ONE, beta, native.MIOC_ALGO_PYRAMID)
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
    du = torch.empty_like(ddf)
    dphi = torch.empty(K, dtype=torch.float64, device="cuda")
    dst = torch.empty(K, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.bellman_batch_tensors(ddf, duo, B, dt)
    ctx.backtrack_batch_tensors(B, du, dphi, dst)
    ctx.synchronize()
    assert ctx.last_algo() == native.MIOC_ALGO_PYRAMID
    ub = du.cpu().numpy()
    for k in range(K):
        single = _ctx(lt, P_ONE, beta, native.MIOC_ALGO_PYRAMID)
        single.bellman(dfs[k], uos[k], B, dt)
        u, ps, _ = single.backtrack(B)
        assert np.array_equal(ub[k].T, u) and dphi[k].item() == ps and dst[k].item() == 0, f"k={k}"
        phi, U = oracle_c.bellman(lv, dfs[k], uos[k], B, P_ONE, beta, dt)
        for i in range(nt - 1):  # every cell the reference writes
            d, o = ctx.argmin_table(i, k=k), U[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"k={k} step {i}"
        single.close()
    ctx.close()


def test_batch_tensor_api_rejects_strided_inputs():
    """np.stack of transposed views is Fortran-ordered and torch.tensor keeps those strides: the raw
    pointer would address a permuted layout, so the tensor API must refuse it."""
    import torch
    lt = LevelTable([[0, 1, 2]] * 2)
    ctx = _ctx(lt, P_ONE, 0.1, native.MIOC_ALGO_GENERIC)
    d = np.zeros((2, 5))
    bad = torch.tensor(np.stack([d.T]), dtype=torch.float64, device="cuda")
    assert not bad.is_contiguous()
    with pytest.raises(ValueError):
        ctx.bellman_batch_tensors(bad, bad, 2, 0.1)
    good = bad.contiguous()
    ctx.bellman_batch_tensors(good, good, 2, 0.1)
    ctx.close()


def test_batch_device_api_equals_single():
    import torch
    cfg = CONFIGS["C5"]
    K, nt, B = 6, 300, 40
    lt = cfg.levels()
    dfs, uos = [], []
    for k in range(K):
        _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=lt)
        dfs.append(df)
        uos.append(uo)
    for pk, algos in ((P_ONE, (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_FUSED, native.MIOC_ALGO_FUSED_SEPARABLE)),
                      (P_INF, ALGOS_PINF + (native.MIOC_ALGO_FUSED,))):
        for algo in algos:
            ctx = _ctx(lt, pk, cfg.beta, algo)
            ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
            duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
            du = torch.empty_like(ddf)
            dphi = torch.empty(K, dtype=torch.float64, device="cuda")
            dst = torch.empty(K, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            ctx.bellman_batch_device(K, ddf.data_ptr(), duo.data_ptr(), lt.M, nt, B, cfg.dt)
            ctx.backtrack_batch_device(B // 2, du.data_ptr(), dphi.data_ptr(), dst.data_ptr())
            ctx.synchronize()
            ub = du.cpu().numpy()
            for k in range(K):
                single = _ctx(lt, pk, cfg.beta, algo)
                single.bellman(dfs[k], uos[k], B, cfg.dt)
                u, ps, _ = single.backtrack(B // 2)
                assert np.array_equal(ub[k].T, u), f"k={k} pk={pk} algo={algo}"
                assert dphi[k].item() == ps and dst[k].item() == 0
                single.close()
            ctx.close()


def test_error_codes():
    lt = LevelTable([[0, 1, 2]])
    ctx = _ctx(lt, P_ONE, 0.1, native.MIOC_ALGO_AUTO)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.backtrack(1)
    assert e.value.code == native.MIOC_ESTATE
    with pytest.raises(native.InexactError):
        ctx.bellman(np.zeros((1, 4)), np.array([[0.0, 0.5, 1.0, 2.0]]), 3, 0.1)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.bellman(np.array([[0.0, np.nan, 1.0, 2.0]]), np.zeros((1, 4)), 3, 0.1)
    assert e.value.code == native.MIOC_ENONFINITE
    with pytest.raises(native.MiocNativeError) as e:
        ctx.bellman(np.zeros((2, 4)), np.zeros((2, 4)), 3, 0.1)
    assert e.value.code == native.MIOC_EINVAL
    ctx.bellman(np.ones((1, 4)), np.zeros((1, 4)), 3, 0.1)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.backtrack(4)
    assert e.value.code == native.MIOC_ESTATE
    # u_old outside every level with budget 0: no finite Φ -> infeasible (the reference reads stale U)
    ctx.bellman(np.ones((1, 4)), np.full((1, 4), 7.0), 0, 0.1)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.backtrack(0)
    assert e.value.code == native.MIOC_EINFEASIBLE
    with pytest.raises(native.MiocNativeError) as e:  # U has nt-1 steps
        ctx.argmin_table(3)
    assert e.value.code == native.MIOC_EINVAL
    ctx.close()
    # the p=Inf collapse keeps class tables, not U
    ctx = _ctx(lt, P_INF, 0.1, native.MIOC_ALGO_PINF)
    ctx.bellman(np.ones((1, 4)), np.zeros((1, 4)), 3, 0.1)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.argmin_table(0)
    assert e.value.code == native.MIOC_EINVAL
    ctx.close()
    # the L1-ball pyramid is exact only for a non-decreasing switching cost (beta >= 0)
    lt2 = LevelTable([list(range(4))] * 2)
    ctx = _ctx(lt2, P_ONE, -0.1, native.MIOC_ALGO_PYRAMID)
    with pytest.raises(native.MiocNativeError) as e:
        ctx.bellman(np.ones((2, 4)), np.zeros((2, 4)), 3, 0.1)
    assert e.value.code == native.MIOC_EINVAL
    ctx.close()


def test_trm_on_gpu_matches_trm_on_oracle():
    """TRM driver end to end (fishing, p=Inf and doubletank-shaped p=1): GPU solver == oracle solver."""
    import mioc
    from mioc.ode import DTMObj, LVMObj
    from test_host import OracleSolver
    for cls, p, beta, D0 in ((LVMObj, math.inf, 1e-4, 2.0), (DTMObj, 1, 1e-3, 0.5)):
        objs = [cls(nt=256), cls(nt=256)]
        par = mioc.TRM_parameters(beta=beta, Delta0=D0, p=p, maxiter=20)
        x0 = mioc.rand_func(objs[0], rng=11)
        lt = LevelTable(objs[0].V, objs[0].iterator)
        J_gpu = mioc.TRM(objs[0], par, x0=x0)
        J_cpu = mioc.TRM(objs[1], par, x0=x0, solver=OracleSolver(lt, p, beta))
        assert J_gpu == J_cpu
        assert np.array_equal(objs[0].x, objs[1].x)


@pytest.mark.parametrize("algo", ["pyramid", "separable", "separable_steps"])
@pytest.mark.parametrize("mode", ["gauss", "integer", "zero", "dyadic", "steep", "outside"])
def test_pyramid_vs_oracle_512_levels(oracle_c, mode, algo):
    """8x8x8 product grid, p=1: clean rows (pyramid + value lookup / certified transform argmin) and
    dirty rows (exact scan).  "steep": value spread ~1e14 times beta, outside the separable
    transform's binade, so its rows go to the exact scan."""
    persist = algo != "separable_steps"
    algo = {"pyramid": native.MIOC_ALGO_PYRAMID, "separable": native.MIOC_ALGO_SEPARABLE,
            "separable_steps": native.MIOC_ALGO_SEPARABLE}[algo]
    rng = np.random.default_rng({"gauss": 1, "integer": 2, "zero": 3, "dyadic": 4, "steep": 5, "outside": 6}[mode])
    lv = Levels.product([list(range(8))] * 3)
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    n, B = 12, 20
    if mode == "gauss":
        df = rng.standard_normal((3, n))
    elif mode == "integer":
        df = rng.integers(-3, 4, size=(3, n)).astype(float)
    elif mode == "zero":
        df = np.zeros((3, n))
    elif mode == "steep":
        df = rng.standard_normal((3, n)) * 1e3
    else:
        df = rng.integers(-64, 65, size=(3, n)) / 64.0
    uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(n)], dtype=np.float64).T
    if mode == "outside":  # u_old off the level grid (integral, not admissible): b̃ beyond the 7·M window
        df = rng.standard_normal((3, n))
        for i in rng.choice(n, size=5, replace=False):
            uo[:, i] = [-1.0, 8.0, 3.0][: 3]
    beta, dt = {"gauss": (1e-3, 2.0 ** -10), "steep": (1e-12, 2.0 ** -10),
                "outside": (1e-3, 2.0 ** -10)}.get(mode, (0.125, 0.25))
    phi, U = oracle_c.bellman(lv, df, uo, B, P_ONE, beta, dt)
    ctx = _ctx(lt, P_ONE, beta, algo)
    ctx.set_option(native.MIOC_OPT_PERSIST, int(persist))
    ctx.bellman(df, uo, B, dt)
    diag = ctx.diagnostics()
    _assert_U(ctx, U, n, mode)
    for Bp in (B, B // 2, 3):
        try:
            ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
        except Exception:  # no finite value within B' (off-grid u_old costs budget at every such step)
            with pytest.raises(native.MiocNativeError):
                ctx.backtrack(Bp)
            continue
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou), f"{mode} Bp={Bp} diag={diag}"
        assert ps == ops
    assert ctx.last_algo() == algo
    if mode in ("integer", "zero"):
        assert diag[0] > 0  # the exact scan for targets whose winning value is tied was exercised
    if algo == native.MIOC_ALGO_SEPARABLE:
        assert diag[1] > 0  # rows near B (few targets) went straight to the exact scan
        if mode == "steep":
            assert diag[0] == 0 and diag[1] > 1000  # every row out of the binade: all exact scans
    ctx.close()


@pytest.mark.parametrize("pk", [P_ONE, P_INF])
@pytest.mark.parametrize("uo_mode", ["piecewise", "random", "outside"])
def test_run_ahead_walk_vs_oracle(oracle_c, uo_mode, pk):
    """Backtrack chains several 64-step rounds long, on and off the walk's two guesses (keep the level;
    follow u_old): u_old piecewise constant, a new random level every step, and partly outside the
    level grid (integral but not admissible, so there is no u_old level to follow)."""
    rng = np.random.default_rng({"piecewise": 11, "random": 12, "outside": 13}[uo_mode] + 10 * (pk == P_INF))
    lv = Levels.product([list(range(4))] * 3)
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    n, B, beta, dt = 333, 24, 1e-3, 2.0 ** -6
    df = rng.standard_normal((3, n))
    if uo_mode == "piecewise":
        idx = np.repeat(rng.integers(lv.L, size=n // 10 + 1), 10)[:n]
    else:
        idx = rng.integers(lv.L, size=n)
    uo = np.array([lv.nuval[j] for j in idx], dtype=np.float64).T.copy()
    if uo_mode == "outside":
        for i in rng.choice(n, size=12, replace=False):
            uo[rng.integers(3), i] = float(rng.choice([-1, 4]))
    phi, U = oracle_c.bellman(lv, df, uo, B, pk, beta, dt)
    for algo in _algos(pk, lt, B):
        ctx = _ctx(lt, pk, beta, algo)
        ctx.bellman(df, uo, B, dt)
        for Bp in (B, B // 3, 0):
            try:
                ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
            except Exception:
                with pytest.raises(native.MiocNativeError):
                    ctx.backtrack(Bp)
                continue
            u, ps, _ = ctx.backtrack(Bp)
            d = ctx.diagnostics()
            assert np.array_equal(u, ou), f"{uo_mode} algo={algo} Bp={Bp} diag={d}"
            assert ps == ops
            assert d[3] == 0
            if algo != native.MIOC_ALGO_PINF:
                assert math.ceil((n - 1) / 64) <= d[2] <= n - 1, d
        ctx.close()


def test_pyramid_equals_generic_at_c4_scale():
    """4096 levels, B=256, p=1: the pyramid, the separable transform and the generic sweep are independent
    algorithms.  Also every U cell of a late step (where most cells are finite) agrees."""
    cfg = CONFIGS["C4"]
    lt, df, uo = make_inputs(cfg, nt=48)
    out, tabs = {}, {}
    algos = (native.MIOC_ALGO_GENERIC, native.MIOC_ALGO_PYRAMID, native.MIOC_ALGO_SEPARABLE, -1)
    for algo in algos:  # -1: the separable transform, one launch per step
        ctx = _ctx(lt, P_ONE, cfg.beta, abs(algo) if algo > 0 else native.MIOC_ALGO_SEPARABLE)
        ctx.set_option(native.MIOC_OPT_PERSIST, int(algo != -1))
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        algo = algo if algo > 0 else -1
        assert ctx.last_algo() == (algo if algo > 0 else native.MIOC_ALGO_SEPARABLE)
        tabs[algo] = [ctx.argmin_table(i) for i in (0, 20, 46)]
        out[algo] = [ctx.backtrack(Bp)[:2] for Bp in (cfg.B, 100, 7)]
        ctx.close()
    for algo in algos[1:]:
        for (ug, pg), (up, pp) in zip(out[native.MIOC_ALGO_GENERIC], out[algo]):
            assert np.array_equal(ug, up) and pg == pp, f"algo={algo}"
    # cells with c >= b̃ that generic and the staged algorithms both wrote agree wherever both are >= 0
    for other in (native.MIOC_ALGO_SEPARABLE, -1):
        both = 0
        for a_, b_ in zip(tabs[native.MIOC_ALGO_PYRAMID], tabs[other]):
            m = (a_ >= 0) & (b_ >= 0)
            both += m.sum()
            assert np.array_equal(a_[m], b_[m])
        assert both > 0.3 * sum(t.size for t in tabs[other][:2])  # the late steps near the terminal are sparse
