"""GPU parity of the p=Inf segmented walk (mioc_pinf.hip, k_pinf_ftab / k_pinf_fseg / k_pinf_fexpand).

The segmented walk replaces the serial forward walk of eval_u_TRM! (multi-trust.jl:104-126, the p=Inf collapse of
DESIGN.md §3.3) by a class table whose entries do not depend on the walker's state, composed over segments of steps.
Bar: controls and Φ* bit-identical to the oracle (small cases) and to the serial walk (full sizes); rows whose
decision could depend on rounding send the subproblem to the serial walk, which the tie-heavy cases exercise.
"""
import numpy as np
import pytest

from mioc import native
from mioc.iterators import LevelTable
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_INF, Levels
from test_gpu_parity import _random_case

pytestmark = pytest.mark.gpu


def _ctx(lt, beta, walk):
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(None, beta, p_kind=P_INF)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_PINF)
    ctx.set_option(native.MIOC_OPT_PINF_WALK, walk)
    return ctx


@pytest.mark.parametrize("seed", range(36))
def test_segmented_walk_vs_oracle(oracle_c, seed):
    """Random small problems (all-zero, integer and Gaussian gradients), forced segmented walk == oracle."""
    lv, df, uo, B, rng = _random_case(2 * seed + 1)
    beta = [1e-3, 0.25, 0.1][seed % 3]
    dt = [0.5, 1 / 3, 2.0 ** -6][seed % 3]
    phi, U = oracle_c.bellman(lv, df, uo, B, P_INF, beta, dt)
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    ctx = _ctx(lt, beta, 1)
    ctx.bellman(df, uo, B, dt)
    for Bp in sorted({B, B // 2, 0}):
        try:
            ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
        except Exception:
            with pytest.raises(native.MiocNativeError):
                ctx.backtrack(Bp)
            continue
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou), f"seed={seed} Bp={Bp}"
        assert ps == ops
        d = ctx.diagnostics()
        assert d[3] == 0 and d[9] in (0, 1), d
    ctx.close()


@pytest.mark.parametrize("key", ["C1", "C2", "C3"])
def test_segmented_walk_sos1_full_size_vs_oracle(oracle_c, key):
    cfg = CONFIGS[key]
    lt, df, uo = make_inputs(cfg)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_INF, cfg.beta, cfg.dt)
    ctx = _ctx(lt, cfg.beta, 1)
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    for Bp in (cfg.B, cfg.B // 2, cfg.B // 8):
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, Bp)
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou) and ps == ops, f"{key} Bp={Bp}"
        assert ctx.diagnostics()[9] == 0  # Gaussian gradients: no state-dependent row on the path
    ctx.close()


@pytest.mark.parametrize("mode", ["gauss", "integer"])
def test_segmented_walk_c4_equals_serial(mode):
    """C4 at full size (4096 levels, nt = 65536, B = 256): the segmented walk and the serial walk agree on
    every control and on Φ*; integer gradients (exact ties everywhere) must fall back to the serial walk."""
    cfg = CONFIGS["C4"]
    lt, df, uo = make_inputs(cfg)
    if mode == "integer":
        df = np.round(df * 4.0)
    out = {}
    for walk in (-1, 1):
        ctx = _ctx(lt, cfg.beta, walk)
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        for Bp in (cfg.B, cfg.B // 3):
            u, ps, _ = ctx.backtrack(Bp)
            out[(walk, Bp)] = (u, ps, ctx.diagnostics())
        ctx.close()
    for Bp in (cfg.B, cfg.B // 3):
        us, pss, ds = out[(-1, Bp)]
        uf, pf, df_ = out[(1, Bp)]
        assert np.array_equal(us, uf) and pss == pf, f"{mode} Bp={Bp}"
        assert ds[9] == -1 and df_[9] in (0, 1) and df_[3] == 0
        if mode == "gauss":
            assert df_[9] == 0, df_


def test_segmented_walk_batch_equals_single():
    """K = 5 subproblems through the batch API (auto: segmented for K <= 64 and nt >= 512), one whose level costs
    is state-dependent (serial fallback for that subproblem only): each equals its serial single run.
    (Exact ties, e.g. a zero gradient, are state-independent and stay on the segmented walk.)"""
    import torch

    cfg = CONFIGS["C2"]
    K, nt = 5, 1024
    lt = None
    dfs, uos = [], []
    for k in range(K):
        lt, df, uo = make_inputs(cfg, nt=nt, k=k)
        if k == 2:  # one huge step cost, then tiny ones: the next rows depend on the state (see below)
            df = df * 1e-10
            df[0, 0] = -1e6
        dfs.append(df)
        uos.append(uo)
    B = cfg.B
    dev = torch.device("cuda:0")
    df_t = torch.tensor(np.stack([d.T for d in dfs]), dtype=torch.float64, device=dev).contiguous()
    uo_t = torch.tensor(np.stack([u.T for u in uos]), dtype=torch.float64, device=dev).contiguous()
    ctx = _ctx(lt, cfg.beta, 0)
    ub = torch.empty_like(df_t)
    pb = torch.empty(K, dtype=torch.float64, device=dev)
    st = torch.empty(K, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the library runs on its own stream
    ctx.bellman_batch_tensors(df_t, uo_t, B, cfg.dt)
    ctx.backtrack_batch_tensors(B, ub, pb, st)
    ctx.synchronize()
    ub, pb, st = ub.cpu().numpy(), pb.cpu().numpy(), st.cpu().numpy()
    for k in range(K):
        c1 = _ctx(lt, cfg.beta, -1)
        c1.bellman(dfs[k], uos[k], B, cfg.dt)
        u, ps, _ = c1.backtrack(B)
        assert st[k] == 0
        assert np.array_equal(ub[k].T, u) and pb[k] == ps, f"k={k}"
        c1.close()
    assert ctx.diagnostics()[9] == 1
    ctx.close()


def test_segmented_walk_state_dependent_rows_vs_oracle(oracle_c):
    """A step whose level costs are ~1e6 followed by steps whose class values differ by ~1e-10: fl(K_l + V_b) then
    collapses classes for the large K_l of the walker's level, so which classes match depends on the state.  The
    class table must mark those rows, the subproblem must go to the serial walk, and the result equal the oracle."""
    rng = np.random.default_rng(7)
    lv = Levels.product([[0, 1, 2, 3]])
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    n, B, beta, dt = 600, 40, 1e-3, 1.0
    df = rng.standard_normal((1, n)) * 1e-10
    df[0, 0] = -1e6
    uo = np.zeros((1, n))
    phi, U = oracle_c.bellman(lv, df, uo, B, P_INF, beta, dt)
    ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, B)
    for walk in (0, 1):
        ctx = _ctx(lt, beta, walk)
        ctx.bellman(df, uo, B, dt)
        u, ps, _ = ctx.backtrack(B)
        assert np.array_equal(u, ou) and ps == ops, f"walk={walk}"
        assert ctx.diagnostics()[9] == 1
        ctx.close()


def _c4_pinf_fixture():
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "hashed", "c4_4096lv_pinf_nt200.npz")
    return np.load(path, allow_pickle=False)


@pytest.mark.parametrize("walk", [1, -1], ids=["segmented_walk", "serial_walk"])
@pytest.mark.parametrize("spin", [0, 1], ids=["run", "timeout_redo"])
def test_c4_pinf_nt200_fixture(walk, spin):
    """C4 at p = Inf (4096 levels, B = 256) over 199 recursion steps against the C oracle's fixture
    (tests/golden/make_c4_pinf_fixture.py): the row-segment recursion k_pinf_recur_mc across more than three of its
    64-step hand-off chunks and a wrap of its 128-slot ring, then u and Φ* at five budgets.  spin = 1: a spin limit of
    one poll abandons the segmented launch at its first unmet wait, and the one-workgroup recursion, launched behind it
    gated by its error word, redoes the DP on the device (diagnostics [6]) before anything reads the tables -- the same
    u and Φ*."""
    z = _c4_pinf_fixture()
    lt = CONFIGS["C4"].levels()
    ctx = _ctx(lt, float(z["beta"][0]), walk)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    if spin:
        ctx.set_option(native.MIOC_OPT_SPIN_LIMIT, 1)
    ctx.bellman(z["df"], z["u_old"], int(z["B"][0]), float(z["dt"][0]))
    ctx.synchronize()
    # the row-segment kernel took this DP (after an abandoned launch its gated one-workgroup redo ran behind it)
    assert ctx.kernel_stats(0)[2] == "k_pinf_recur_mcw"
    for q, Bp in enumerate(z["budgets"]):
        u, ps, _ = ctx.backtrack(int(Bp))
        assert np.array_equal(u, z["u"][q]), f"B'={Bp}"
        assert ps == z["phi_star"][q], f"B'={Bp}: {ps!r} vs {z['phi_star'][q]!r}"
    diag = ctx.diagnostics()
    if spin:
        assert diag[6] >= 1, diag  # the segmented launch was abandoned and redone
    else:
        assert diag[6] == 0, diag
    ctx.close()
