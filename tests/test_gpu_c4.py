"""GPU parity of the C4 (BASELINE roofline) shape on the code the bench times: k_sdt_run<4> (the persistent separable
transform, one workgroup per budget row, 8^4 = 4096 levels, B = 256, p = 1) -- and the per-step k_sdt_step --
against the CPU oracle, never against another device algorithm.

  * a committed oracle fixture at the full L = 4096, B = 256 with nt = 64 (63 recursion steps and row B's two-step
    lag): sha256 of every step's argmin table U in the reference layout, and u / Φ* at B' = 256, 128, 7
    (tests/golden/make_c4_fixture.py).  At the default 256 staging buffers a 63-step DP never reuses one, so the
    fixture also runs with 29 (the fewest that cannot deadlock: 7·M + 1), 32 and 37 buffers (MIOC_OPT_SDT_BUFFERS):
    the ring wraps and every row below B arms its write-after-read wait on the rows above for nt - NB steps
    (diagnostics [4] counts those rows); 4 is raised to 29;
  * 4096-level tie-heavy steps (zero, integer, steep gradients): the exact-scan paths, including the overflow
    of the listed-target buffer (SD_LCAP), oracle computed here;
  * the chunked persistent branch (each workgroup several rows): a K = 2 batch and B = 300 > #CUs.
"""
import hashlib
import os

import numpy as np
import pytest

from mioc import native
from mioc.iterators import LevelTable
from mioc.synth import CONFIGS, make_inputs
from oracle.oracle import P_ONE, Levels

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _ctx(lt, beta, algo, persist=1, nb=None):
    ctx = native.Context(0)
    ctx.set_levels(lt)
    ctx.set_cost(1, beta)
    if nb is not None:
        ctx.set_option(native.MIOC_OPT_SDT_BUFFERS, nb)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    ctx.set_option(native.MIOC_OPT_ALGO, algo)
    ctx.set_option(native.MIOC_OPT_PERSIST, persist)
    return ctx


def _hash(t):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(t, dtype=np.int32).tobytes()).digest(), dtype=np.uint8)


# (variant, staging buffers): None = the default (256, no reuse at nt = 64); 29 / 32 / 37 wrap the ring (29 and 37 are
# not powers of two, so an off-by-one in the buffer index that a power of two would hide cannot pass); 4 is below the
# deadlock-free minimum 7·M + 1 = 29 and must be raised to it
C4_VARIANTS = [("persistent", None), ("persistent", 29), ("persistent", 32), ("persistent", 37), ("persistent", 4),
               ("steps", None)]
NB_MIN = 29


def _check_fixture(ctx, z, label):
    nt = z["df"].shape[1]
    bad = [i for i in range(nt - 1) if not np.array_equal(_hash(ctx.argmin_table(i)), z["u_hash"][i])]
    assert not bad, f"{label}: U differs from the oracle at steps {bad[:10]}"
    for q, Bp in enumerate(z["budgets"]):
        u, ps, _ = ctx.backtrack(int(Bp))
        assert np.array_equal(u, z["u"][q]), f"{label} B'={Bp}"
        assert ps == z["phi_star"][q], f"{label} B'={Bp}: {ps!r} vs {z['phi_star'][q]!r}"


@pytest.mark.parametrize("variant,nb", C4_VARIANTS, ids=[f"{v}-nb{n}" if n else v for v, n in C4_VARIANTS])
def test_c4_nt64_fixture(variant, nb):
    """The separable transform writes U exactly like the reference: the rank where the reference writes it, and
    nothing (-1) elsewhere, so every step's table hashes to the oracle's.  persistent: k_sdt_run (the bench's kernel),
    steps: one k_sdt_step launch per step.  With nb staging buffers the ring wraps and the WAR waits run."""
    z = np.load(os.path.join(HERE, "golden", "hashed", "c4_4096lv_p1_nt64_uhash.npz"), allow_pickle=False)
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    algo = native.MIOC_ALGO_SEPARABLE
    ctx = _ctx(lt, float(z["beta"][0]), algo, persist=int(variant != "steps"), nb=nb)
    df, uo = z["df"], z["u_old"]
    B = int(z["B"][0])
    ctx.bellman(df, uo, B, float(z["dt"][0]))
    assert ctx.last_algo() == algo
    ctx.synchronize()
    assert ctx.kernel_stats(0)[2] == {"persistent": "k_sdt_run", "steps": "k_sdt_step"}[variant]
    diag = ctx.diagnostics()
    assert diag[6] == 0, diag  # the persistent launch ran to the end (no per-step redo)
    if variant == "persistent":
        nt = df.shape[1]
        if nb is None:
            assert diag[4] == 0, diag  # 256 buffers, 63 steps: no buffer is reused
        else:
            # one row per workgroup: rows 1 .. B-1 arm the WAR wait at every step i < nt - NB (token(i + NB - 1) > 0)
            assert diag[4] == (B - 1) * (nt - max(nb, NB_MIN)), diag
    _check_fixture(ctx, z, f"{variant} nb={nb}")
    ctx.close()


@pytest.mark.parametrize("variant", ["persistent", "steps"])
@pytest.mark.parametrize("mode", ["zero", "integer", "steep"])
def test_c4_tie_heavy_vs_oracle(oracle_c, mode, variant):
    """4096 levels, B = 256: every target of a zero-gradient row ties (the listed-target buffer overflows and the
    scan sweeps every rank); integer gradients tie often; 'steep' puts rows outside the transform's binade."""
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    rng = np.random.default_rng({"zero": 31, "integer": 32, "steep": 33}[mode])
    n = 3
    _, df, uo = make_inputs(cfg, nt=n, levels=lt)
    if mode == "zero":
        df = np.zeros_like(df)
    elif mode == "integer":
        df = rng.integers(-3, 4, size=df.shape).astype(float) * 4096.0
    elif mode == "steep":
        df = df * 1e3  # value spread ~1e12 beta: outside the transform's binade (2^36 units)
    beta = 1e-13 if mode == "steep" else cfg.beta
    phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_ONE, beta, cfg.dt)
    ctx = _ctx(lt, beta, native.MIOC_ALGO_SEPARABLE, int(variant != "steps"))
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    diag = ctx.diagnostics()
    for i in range(n - 1):
        d, o = ctx.argmin_table(i), U[:, :, i]
        m = o >= 0
        assert np.array_equal(d[m], o[m]), f"{mode} step {i}"
    for Bp in (cfg.B, 100, 3):
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, Bp)
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou) and ps == ops, f"{mode} B'={Bp} diag={diag}"
    if mode == "zero":
        assert diag[0] > 2 * 512, diag  # rows with more tied targets than the list holds: the full-rank sweep
    if mode == "steep":
        assert diag[1] > 1000, diag     # rows outside the binade: exact scans
    ctx.close()


def test_c4_chunked_rows_vs_oracle(oracle_c):
    """The persistent kernel with several rows per workgroup: a K = 2 batch (128 workgroups per subproblem) and
    one subproblem with B = 300 (301 rows on the CUs), each against the oracle."""
    import torch
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    lv = Levels(lt.nu, [tuple(int(x) for x in t) for t in lt.tuples])
    n = 4
    subs = [make_inputs(cfg, k=k, nt=n, levels=lt)[1:] for k in (7, 8)]
    ctx = _ctx(lt, cfg.beta, native.MIOC_ALGO_SEPARABLE, 1)
    ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d, _ in subs])), dtype=torch.float64, device="cuda")
    duo = torch.tensor(np.ascontiguousarray(np.stack([u.T for _, u in subs])), dtype=torch.float64, device="cuda")
    du = torch.empty_like(ddf)
    dphi = torch.empty(2, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    ctx.backtrack_batch_tensors(cfg.B, du, dphi, None)
    ctx.synchronize()
    assert ctx.kernel_stats(0)[2] == "k_sdt_run"
    for k, (df, uo) in enumerate(subs):
        phi, U = oracle_c.bellman(lv, df, uo, cfg.B, P_ONE, cfg.beta, cfg.dt)
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, cfg.B, cfg.B)
        assert np.array_equal(du[k].cpu().numpy().T, ou) and dphi[k].item() == ops, f"batch k={k}"
        for i in range(n - 1):
            d, o = ctx.argmin_table(i, k=k), U[:, :, i]
            m = o >= 0
            assert np.array_equal(d[m], o[m]), f"batch k={k} step {i}"
    ctx.close()
    B = 300
    df, uo = subs[0]
    phi, U = oracle_c.bellman(lv, df, uo, B, P_ONE, cfg.beta, cfg.dt)
    ctx = _ctx(lt, cfg.beta, native.MIOC_ALGO_SEPARABLE, 1)
    ctx.bellman(df, uo, B, cfg.dt)
    for Bp in (B, 150):
        ou, ops = oracle_c.backtrack(lv, uo, phi, U, B, Bp)
        u, ps, _ = ctx.backtrack(Bp)
        assert np.array_equal(u, ou) and ps == ops, f"B=300 B'={Bp}"
    ctx.close()


@pytest.mark.parametrize("nb", [None, 31], ids=["nb-default", "nb31"])
def test_c4_nt64_fixture_wait_timeout_redoes_dp(nb):
    """The headline kernel's timeout path: with a spin limit of one poll, the persistent k_sdt_run gives up at its
    first dependency wait that is not already satisfied (RAW, or with 31 staging buffers also WAR), every workgroup
    leaves, and the host redoes the DP with per-step launches (check_run, counted in diagnostics [6]) before anything
    reads the tables -- so every step's U hash, u and Φ* still equal the oracle fixture."""
    z = np.load(os.path.join(HERE, "golden", "hashed", "c4_4096lv_p1_nt64_uhash.npz"), allow_pickle=False)
    lt = CONFIGS["C4"].levels()
    algo = native.MIOC_ALGO_SEPARABLE
    ctx = _ctx(lt, float(z["beta"][0]), algo, persist=1, nb=nb)
    ctx.set_option(native.MIOC_OPT_SPIN_LIMIT, 1)
    df, uo = z["df"], z["u_old"]
    ctx.bellman(df, uo, int(z["B"][0]), float(z["dt"][0]))
    assert ctx.last_algo() == algo
    _check_fixture(ctx, z, f"timeout redo nb={nb}")
    diag = ctx.diagnostics()
    assert diag[6] >= 1, diag  # the persistent launch was abandoned and redone
    ctx.close()
