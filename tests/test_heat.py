"""The PDE heat objective: oracle checks on CPU, device parity on the GPU.

CPU tier: the oracle (oracle/heat_oracle.py, LU restatement of julia_opt/PDEObjective.jl:129-199) is pinned the way
the reference checks its own gradient -- example_heat.jl:186-223 (test_df) compares τ·Σ df·h with finite differences
of eval_f -- here as a convergence statement: on a smooth direction vanishing at both ends the mismatch is O(τ) and
halves when nt doubles (a wrong step index, sign or factor would leave it at O(1)).  Plus the stand-in assembly's
invariants (mass of the square = 4, constant state0).

GPU tier: mioc_heat_eval_device against the oracle on the same matrices.  Bar: |J − J_oracle| ≤ 1e-9·|J_oracle| and
max|df − df_oracle| ≤ 1e-9·max|df_oracle| (the device multiplies by the precomputed inverse of StateMat on the FP64
matrix cores; the reference solves with its LU factors, so the results agree to rounding, not bit for bit).
N <= 512 keeps the 16 state columns in LDS, larger N (up to 2048) in a global scratch: both are covered.
"""
import os

import numpy as np
import pytest

from mioc.heat import HeatProblem
from oracle.heat_oracle import HeatOracle


def _oracle(hp):
    return HeatOracle(hp.M_invA, hp.M_invF, hp.M, hp.state0, hp.yd, hp.T0, hp.T1, hp.gamma)


HEAT_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "heat", "heat_n5_nt24.npz")


def _golden():
    z = np.load(HEAT_GOLDEN, allow_pickle=False)
    return {k: z[k] for k in z.files}


def test_oracle_reproduces_heat_golden():
    """The committed fixture (tests/golden/heat/make_heat_golden.py): the oracle on its stored matrices reproduces
    J and df to 1e-12 relative (a regression anchor for the restatement; bit-equal on the machine that wrote it,
    LAPACK builds elsewhere may round the triangular solves differently)."""
    g = _golden()
    T0, T1, gamma = g["scalars"]
    o = HeatOracle(g["M_invA"], g["M_invF"], g["M"], g["state0"], g["yd"], T0, T1, gamma)
    for k in range(len(g["x"])):
        f, df, _ = o.eval(g["x"][k])
        assert abs(f - g["J"][k]) <= 1e-12 * abs(g["J"][k]), k
        assert np.max(np.abs(df - g["df"][k])) <= 1e-12 * np.max(np.abs(g["df"][k])), k


def test_standin_assembly_invariants():
    hp = HeatProblem(n=9, nt=10)
    assert hp.N == 81
    assert abs(hp.M.sum() - 4.0) < 1e-12                       # ∫_Ω 1 = |[-1,1]²|
    assert np.allclose(hp.M, hp.M.T) and np.allclose(hp.A, hp.A.T)
    assert np.max(np.abs(hp.state0 - 10.0)) < 1e-12            # y0 = temp0
    assert abs(hp.A.sum() - 0.12 * 8.0) < 1e-12                 # Robin κ·|Γ| (the Laplacian part sums to 0)


def test_oracle_gradient_is_first_order_consistent():
    errs = []
    for nt in (100, 200, 400):
        hp = HeatProblem(n=9, nt=nt)
        o = _oracle(hp)
        u = np.ones((2, nt))
        f0, df, _ = o.eval(u)
        s = np.linspace(0.0, 1.0, nt)
        h = np.vstack([np.sin(np.pi * s) ** 2, np.sin(2 * np.pi * s) ** 2])
        dfh = o.tau * np.sum(df * h)                            # example_heat.jl:204-209
        t = 1e-5
        f1, _, _ = o.eval(u + t * h)
        errs.append(abs((f1 - f0) / t - dfh) / abs(dfh))
    assert errs[0] < 1e-2
    for a, b in zip(errs, errs[1:]):
        assert 0.4 < b / a < 0.6, errs                           # O(τ)


def test_oracle_stationary_cost():
    """u = 0, Tout = 0: the state decays from temp0; with yd = temp0 the first trapezoid term is 0 and J only has
    the G part.  With γ and a constant control, G_t contributes exactly τ·γ·Σx·nt."""
    hp = HeatProblem(n=5, nt=20, tempT=10.0)
    o = _oracle(hp)
    f0, _, state = o.eval(np.zeros((2, 20)))
    assert abs(o.G(state, 0)) < 1e-20
    # linearity of the state in x: J(x) - J(0) - Gt part is quadratic + linear in x -> check with x and 2x
    x = np.full((2, 20), 1.0)
    fx, _, _ = o.eval(x)
    f2x, _, _ = o.eval(2 * x)
    gt = o.tau * hp.gamma * 2.0 * 20                             # trapezoid of γ·Σx over the extended columns
    # J(cx) = f0 + c·(b + gt) + c²·q  ->  J(2x) - 2 J(x) + f0 = 2q, and the G-only part is consistent
    q = (f2x - 2 * fx + f0) / 2
    b = fx - f0 - q - gt
    f3x, _, _ = o.eval(3 * x)
    assert abs(f3x - (f0 + 3 * (b + gt) + 9 * q)) <= 1e-9 * abs(f3x)


# ---------------------------------------------------------------- GPU parity ---------------------------------------

def _device_eval(hp, xs, want_df=True):
    import torch
    from mioc import native
    ctx = native.Context(0)
    hp.setup(ctx)
    dx = torch.tensor(np.ascontiguousarray(np.stack([x.T for x in xs])), dtype=torch.float64, device="cuda")
    J = torch.empty(len(xs), dtype=torch.float64, device="cuda")
    df = torch.empty_like(dx) if want_df else None
    ctx.heat_eval_tensors(dx, J, df)
    ctx.synchronize()
    out = J.cpu().numpy(), (df.cpu().numpy() if want_df else None)
    ctx.close()
    return out


def _controls(hp, K, seed):
    rng = np.random.default_rng(seed)
    xs = []
    for _ in range(K):  # piecewise-constant integer controls in 𝓥 = 0..5, like rand_func_int
        jumps = np.sort(rng.choice(np.arange(1, hp.nt), size=min(hp.nt - 1, max(1, hp.nt // 10)), replace=False))
        seg = np.searchsorted(jumps, np.arange(hp.nt), side="right")
        lv = rng.integers(0, 6, size=(2, seg.max() + 1)).astype(np.float64)
        xs.append(lv[:, seg])
    return xs


def _check(hp, xs, J, df):
    o = _oracle(hp)
    for k, x in enumerate(xs):
        fo, dfo, _ = o.eval(x)
        assert abs(J[k] - fo) <= 1e-9 * abs(fo), (k, J[k], fo)
        if df is not None:
            assert np.max(np.abs(df[k].T - dfo)) <= 1e-9 * np.max(np.abs(dfo)), k


@pytest.mark.gpu
@pytest.mark.parametrize("n,nt,K", [(17, 500, 20), (5, 64, 33), (2, 7, 3), (22, 40, 16), (9, 1, 5), (12, 2, 17),
                                    (23, 12, 18), (33, 20, 9)],
                         ids=["heat289_nt500", "N25_ragged", "N4", "N484_maxLDS", "nt1", "nt2", "N529_global",
                              "N1089_global"])
def test_heat_eval_device_vs_oracle(n, nt, K):
    hp = HeatProblem(n=n, nt=nt)
    xs = _controls(hp, K, seed=n * 1000 + nt)
    J, df = _device_eval(hp, xs)
    _check(hp, xs, J, df)


@pytest.mark.gpu
@pytest.mark.parametrize("nh", [1, 3, 4], ids=["nx1", "nx3", "nx4"])
def test_heat_control_counts_vs_oracle(nh):
    """1 to 4 heaters (nx, the controls per step; mioc_heat_setup accepts up to 4)."""
    spots = ((-1.0, 0.0), (1.0, 0.0), (0.0, 1.0), (0.0, -1.0))[:nh]
    hp = HeatProblem(n=7, nt=30, c1=(10.0,) * nh, c2=(20.0,) * nh, heaters=spots)
    rng = np.random.default_rng(nh)
    xs = [rng.integers(0, 6, size=(nh, hp.nt)).astype(np.float64) for _ in range(5)]
    J, df = _device_eval(hp, xs)
    _check(hp, xs, J, df)


@pytest.mark.gpu
def test_heat_device_vs_golden():
    """The device on the committed fixture's matrices and controls against its stored J / df (1e-9 relative)."""
    import torch
    from mioc import native
    g = _golden()
    T0, T1, gamma = g["scalars"]
    ctx = native.Context(0)
    ctx.heat_setup(g["M_invA"], g["M_invF"], g["M"], g["state0"], g["yd"], T0, T1, gamma)
    dx = torch.tensor(np.ascontiguousarray(g["x"].transpose(0, 2, 1)), dtype=torch.float64, device="cuda")
    J = torch.empty(len(g["x"]), dtype=torch.float64, device="cuda")
    df = torch.empty_like(dx)
    ctx.heat_eval_tensors(dx, J, df)
    ctx.synchronize()
    J, df = J.cpu().numpy(), df.cpu().numpy()
    ctx.close()
    for k in range(len(g["x"])):
        assert abs(J[k] - g["J"][k]) <= 1e-9 * abs(g["J"][k]), k
        assert np.max(np.abs(df[k].T - g["df"][k])) <= 1e-9 * np.max(np.abs(g["df"][k])), k


@pytest.mark.gpu
def test_heat_J_only_equals_J_with_gradient():
    hp = HeatProblem(n=9, nt=50)
    xs = _controls(hp, 19, seed=3)
    J1, _ = _device_eval(hp, xs, want_df=False)
    J2, _ = _device_eval(hp, xs, want_df=True)
    assert np.array_equal(J1, J2)


@pytest.mark.gpu
def test_heat_batch_restart_independence():
    """1024 restarts (64 workgroups): copies of the same control in different tiles and lanes give bit-identical
    J / df, and a seeded subset matches the oracle."""
    hp = HeatProblem(n=17, nt=100)
    base = _controls(hp, 8, seed=11)
    xs = [base[k % 8] for k in range(1024)]
    J, df = _device_eval(hp, xs)
    for k in range(8, 1024):
        assert J[k] == J[k % 8] and np.array_equal(df[k], df[k % 8]), k
    _check(hp, base, J[:8], df[:8])


@pytest.mark.gpu
def test_heat_host_entry_equals_device_entry():
    """mioc_heat_eval (host arrays, what the Julia binding calls) gives the device entry's results bit for bit."""
    from mioc import native
    hp = HeatProblem(n=9, nt=60)
    xs = _controls(hp, 21, seed=8)
    J, df = _device_eval(hp, xs)
    ctx = native.Context(0)
    hp.setup(ctx)
    Jh, dfh = ctx.heat_eval(np.stack(xs))
    ctx.close()
    assert np.array_equal(Jh, J) and np.array_equal(dfh.transpose(0, 2, 1), df)


@pytest.mark.gpu
def test_heat_errors():
    from mioc import native
    ctx = native.Context(0)
    with pytest.raises(native.MiocNativeError):
        HeatProblem(n=46, nt=2).setup(ctx)  # N = 2116 > 2048
    with pytest.raises(native.MiocNativeError):  # nx = 5 > 4
        ctx.heat_setup(np.eye(4), np.zeros((4, 5)), np.eye(4), np.ones(4), np.ones((4, 3)), 0.0, 1.0, 1.0)
    with pytest.raises(native.MiocNativeError):  # T1 <= T0
        ctx.heat_setup(np.eye(4), np.zeros((4, 2)), np.eye(4), np.ones(4), np.ones((4, 3)), 1.0, 1.0, 1.0)
    import torch
    ctx.heat_shape = (4, 2, 4)
    with pytest.raises(native.MiocNativeError) as e:  # eval before a successful setup
        ctx.heat_eval_tensors(torch.zeros((1, 4, 2), dtype=torch.float64, device="cuda"))
    assert e.value.code == native.MIOC_ESTATE
    ctx.close()


@pytest.mark.gpu
def test_trm_batch_heat_equals_sequential_trm():
    """Multi-start TRM on the heat example entirely on the device (random starts, heat gradient, fused separable DP on
    the 6 x 6 product levels, per-restart budgets, pred, decision) against the host TRM loop (multi-trust.jl:53-170
    mirror) run restart by restart on HeatObj, whose eval_f! / eval_df! call the same heat kernel: identical values
    J + β·TV_p(u) and controls."""
    import math

    import torch

    import mioc
    from mioc import native
    from mioc.heat import HeatObj
    from mioc.iterators import LevelTable
    from mioc.trm_batch import TRM_batch
    hp = HeatProblem(n=9, nt=100)
    K = 6
    par = mioc.TRM_parameters(beta=1e-2, Delta0=2.0, p=1, maxiter=4, kmax=4)
    ctx = native.Context(0)
    ctx.set_levels(LevelTable(hp.levels))
    x0 = torch.empty(K, hp.nt, 2, dtype=torch.float64, device="cuda")
    ctx.rand_start_tensor(x0, seed=5)
    ctx.synchronize()
    log = []
    vals, u, iters = TRM_batch(hp, par, x0=x0, log=log)
    ub = u.cpu().numpy()
    for k in range(K):
        obj = HeatObj(hp)
        J = mioc.TRM(obj, par, x0=x0[k].cpu().numpy().T.copy())
        assert J == vals[k], (k, J, vals[k])
        assert np.array_equal(obj.x, ub[k].T), k
        assert math.isfinite(J)
        obj.ctx.close()
    print(f"heat: iterations per restart {iters.tolist()}, values {vals.tolist()}")
    ctx.close()


@pytest.mark.gpu
def test_trm_batch_heat_reference_config_p2():
    """The reference's own heat run, main("heat") (multi-trust.jl:193-195, example_heat.jl:39,42-44): p = 2,
    β = 1e-3, Δ⁰ = 2, nt = 500 (τ = 0.02, B = 100), 6 x 6 product levels.  TRM_batch (device control, fused DP with
    the p = 2 weight LUT, production path log=None) against the host TRM loop run restart by restart on HeatObj:
    identical values and controls.  The LUT's square roots come from Python's pow here (Julia's ^ supplies them
    through integration/MIOC.jl), so parity with the reference's own floats is unpinned for p = 2."""
    import math

    import torch

    import mioc
    from mioc import native
    from mioc.heat import HeatObj
    from mioc.iterators import LevelTable
    from mioc.trm_batch import TRM_batch
    hp = HeatProblem(n=17, nt=500)
    K = 4
    par = mioc.TRM_parameters(beta=1e-3, Delta0=2.0, p=2, maxiter=3, kmax=4)
    assert math.floor(par.Delta0 / hp.tau) == 100
    ctx = native.Context(0)
    ctx.set_levels(LevelTable(hp.levels))
    x0 = torch.empty(K, hp.nt, 2, dtype=torch.float64, device="cuda")
    ctx.rand_start_tensor(x0, seed=11)
    ctx.synchronize()
    vals, u, iters = TRM_batch(hp, par, x0=x0)
    ub = u.cpu().numpy()
    for k in range(K):
        obj = HeatObj(hp)
        J = mioc.TRM(obj, par, x0=x0[k].cpu().numpy().T.copy())
        assert J == vals[k], (k, J, vals[k])
        assert np.array_equal(obj.x, ub[k].T), k
        assert math.isfinite(J)
        obj.ctx.close()
    print(f"heat p=2: iterations per restart {iters.tolist()}, values {vals.tolist()}")
    ctx.close()
