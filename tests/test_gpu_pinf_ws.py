"""GPU parity of k_pinf_recur_ws (mioc_pinf.hip): the p = Inf recursion R_i[c] = min_b fl(Kmin_i[b] + R_{i+1}[c - b])
for few subproblems with at most 8 budget classes -- the SOS1 shapes of the reference's main() presets
(multi-trust.jl:183-189: fishing, doubletank, vanderpol) -- in 64-row segments on several CUs, the step's chain by DPP
wave shifts.  Bar: u and Φ* bit-identical to the C oracle (HelpFunctions.jl:20-124 restated) at several budgets, the
kernel named in the stats, and the spin-limit redo (one workgroup, check_run) giving the same answer.
"""
import numpy as np
import pytest

from mioc import native
from mioc.iterators import LevelTable
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_INF, Levels

pytestmark = pytest.mark.gpu


def _ctx(lt, beta, spin=0):
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(None, beta, p_kind=P_INF)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_PINF)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    if spin:
        ctx.set_option(native.MIOC_OPT_SPIN_LIMIT, spin)
    return ctx


def _check(oracle_c, lv, lt, df, uo, B, beta, dt, budgets, spin=0):
    phi, U = oracle_c.bellman(lv, df, uo, B, P_INF, beta, dt)
    ctx = _ctx(lt, beta, spin)
    ctx.bellman(df, uo, B, dt)
    ctx.synchronize()
    name = ctx.kernel_stats(0)[2]
    for Bp in budgets:
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou), f"B'={Bp}"
        assert ps == ops, f"B'={Bp}: {ps!r} vs {ops!r}"
    diag = ctx.diagnostics()
    ctx.close()
    return name, diag


@pytest.mark.parametrize("spin", [0, 1], ids=["run", "timeout_redo"])
@pytest.mark.parametrize("key", ["C1", "C2", "C3"])
def test_ws_sos1_full_size_vs_oracle(oracle_c, key, spin):
    """C1-C3 at full size (B + 1 = 86 / 820 / 820 rows: 2 / 13 / 13 segments).  spin = 1: the first unmet wait
    abandons the launch and the one-workgroup recursion launched behind it (gated by the error word) redoes the DP on
    the device before anything reads R."""
    cfg = CONFIGS[key]
    lt, df, uo = make_inputs(cfg)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    name, diag = _check(oracle_c, lv, lt, df, uo, cfg.B, cfg.beta, cfg.dt, (cfg.B, cfg.B // 2, cfg.B // 8, 0), spin)
    if spin:
        assert diag[6] >= 1, diag
    else:
        assert name == "k_pinf_recur_ws", name
        assert diag[6] == 0, diag


@pytest.mark.parametrize("seed", range(24))
def test_ws_random_vs_oracle(oracle_c, seed):
    """Class windows of 2 .. 8 (one- and two-dimensional level grids and SOS1), 2 .. 5 segments, zero / integer /
    Gaussian gradients (exact ties everywhere in the first two)."""
    rng = np.random.default_rng(4000 + seed)
    shapes = [[[0, 1]], [[0, 1, 2]], [list(range(4))], [list(range(5))], [list(range(6))], [list(range(7))],
              [list(range(8))], [[0, 1]] * 3, [list(range(4))] * 2, [[0, 1, 2]] * 2, [[-2, 0, 3]], "sos1"]
    nu = shapes[seed % len(shapes)]
    lv = Levels.bounded_sum([[0, 1]] * 3, 1, 1) if nu == "sos1" else Levels.product(nu)
    lt = LevelTable(lv.nu, [tuple(t) for t in lv.tuples])
    n = int(rng.integers(2, 160))
    B = int(rng.integers(64, 330))
    mode = seed % 3
    if mode == 0:
        df = np.zeros((lv.M, n))
    elif mode == 1:
        df = rng.integers(-4, 5, size=(lv.M, n)).astype(float)
    else:
        df = rng.standard_normal((lv.M, n))
    uo = np.array([lv.nuval[rng.integers(lv.L)] for _ in range(n)], dtype=np.float64).T
    beta = [1e-3, 0.25, 0.1][seed % 3]
    dt = [0.5, 1 / 3, 2.0 ** -6][(seed // 3) % 3]
    budgets = sorted({B, B // 2, 0, int(rng.integers(0, B + 1))})
    name, diag = _check(oracle_c, lv, lt, df, uo, B, beta, dt, budgets)
    assert name == "k_pinf_recur_ws", (name, nu, B)
    assert diag[6] == 0, diag


def test_ws_batch_vs_oracle(oracle_c):
    """K = 3 C2 subproblems through the batch API (3 x 13 segment workgroups), each against the oracle."""
    import torch

    cfg = CONFIGS["C2"]
    K, nt = 3, 1024
    dfs, uos, lt = [], [], None
    for k in range(K):
        lt, df, uo = make_inputs(cfg, nt=nt, k=k)
        dfs.append(df)
        uos.append(uo)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    dev = torch.device("cuda:0")
    df_t = torch.tensor(np.stack([d.T for d in dfs]), dtype=torch.float64, device=dev).contiguous()
    uo_t = torch.tensor(np.stack([u.T for u in uos]), dtype=torch.float64, device=dev).contiguous()
    ctx = _ctx(lt, cfg.beta)
    ub = torch.empty_like(df_t)
    pb = torch.empty(K, dtype=torch.float64, device=dev)
    st = torch.empty(K, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the library runs on its own stream
    ctx.bellman_batch_tensors(df_t, uo_t, cfg.B, cfg.dt)
    ctx.backtrack_batch_tensors(cfg.B, ub, pb, st)
    ctx.synchronize()
    assert ctx.kernel_stats(0)[2] == "k_pinf_recur_ws"
    ub, pb, st = ub.cpu().numpy(), pb.cpu().numpy(), st.cpu().numpy()
    for k in range(K):
        phi, U = oracle_c.bellman(lv, dfs[k], uos[k], cfg.B, P_INF, cfg.beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uos[k], phi, U, cfg.B, cfg.B)
        assert st[k] == 0
        assert np.array_equal(ub[k].T, ou) and pb[k] == ops, f"k={k}"
    ctx.close()


@pytest.mark.parametrize("nt", [65, 129])
def test_ws_full_first_chunk_vs_oracle(oracle_c, nt):
    """nt = 65 and 129 (65 * k: the first, top chunk is full -- (nt - 2) % 64 == 63 -- so the counted-wait path with
    no previous chunk (mid() with prev_lo = -1, then vmcnt(56)) runs from the first chunk on), C2's shape (13
    segments), Gaussian gradients, against the oracle at three budgets."""
    cfg = CONFIGS["C2"]
    lt, df, uo = make_inputs(cfg, nt=nt, k=11)
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    name, diag = _check(oracle_c, lv, lt, df, uo, cfg.B, cfg.beta, cfg.dt, (cfg.B, cfg.B // 3, 5))
    assert name == "k_pinf_recur_ws", name
    assert diag[6] == 0, diag
