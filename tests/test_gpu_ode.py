"""GPU parity of the batched ODE gradient producer: mioc_ode_eval_device against the scalar oracle
oracle/ode_oracle.py (ODEObjective.jl:125-184 with the fishing / doubletank / vanderpol hooks, pinned by the reference's
own finite-difference test_df) and against the product's host mirror (mioc/ode.py).

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
    from oracle.ode_oracle import ODEOracle
    o = ODEOracle(name, nt)
    exact = exact_o = 0
    for k in range(K):
        assert abs(J[k] - Jh[k]) <= 1e-12 * abs(Jh[k]), (k, J[k], Jh[k])
        d, h = df[k].T, dfh[k]
        assert np.max(np.abs(d - h)) <= 1e-12 * max(1e-300, np.max(np.abs(h))), k
        exact += int(J[k] == Jh[k]) + int(np.array_equal(d, h))
        Jo, dfo = o.eval_df([tuple(c) for c in xs[k].T])
        dfo = np.array(dfo).T
        assert abs(J[k] - Jo) <= 1e-12 * abs(Jo), (k, J[k], Jo)
        assert np.max(np.abs(d - dfo)) <= 1e-12 * max(1e-300, np.max(np.abs(dfo))), k
        exact_o += int(J[k] == Jo) + int(np.array_equal(d, dfo))
    print(f"{name}: {exact} of {2 * K} J / df arrays bit-identical to the host mirror, {exact_o} to the oracle")
    ctx.close()


def test_ode_eval_j_only_after_smaller_gradient_call():
    """A J-only call with more restarts / steps than an earlier gradient call (the forward states are stored for
    every restart either way, so the context's state buffer must grow for both: ADVICE r2)."""
    import torch
    from oracle.ode_oracle import ODEOracle
    ctx = native.Context(0)
    obj = _obj("fishing", 64)
    x1 = torch.tensor(np.ascontiguousarray(np.stack([mioc.rand_func(obj, rng=k).T for k in range(4)])),
                      dtype=torch.float64, device="cuda")
    ctx.ode_eval_tensors(native.MIOC_ODE_FISHING, x1, obj.T0, obj.T1, None, torch.empty_like(x1))
    nt, K = 512, 1024
    o = ODEOracle("fishing", nt)
    big = _obj("fishing", nt)
    xs = [mioc.rand_func(big, rng=1000 + k) for k in range(K)]
    x2 = torch.tensor(np.ascontiguousarray(np.stack([x.T for x in xs])), dtype=torch.float64, device="cuda")
    J = torch.empty(K, dtype=torch.float64, device="cuda")
    ctx.ode_eval_tensors(native.MIOC_ODE_FISHING, x2, big.T0, big.T1, J, None)
    ctx.synchronize()
    for k in (0, 517, K - 1):
        Jo = o.eval_f([tuple(c) for c in xs[k].T])
        assert abs(J[k].item() - Jo) <= 1e-12 * abs(Jo), k
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


# ---- rand_func_int on the device (HelpFunctions.jl:204-225) -------------------------------------------------------
_M64 = (1 << 64) - 1


def _mix(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _uniform(key, stream, idx, n):
    v = _mix(key ^ ((stream << 56) & _M64) ^ idx)
    return ((v >> 32) * n) >> 32


def _rand_start_host(levels, nt, jumps, seed, k):
    """Host restatement of k_rand_start's stream (test-only): Floyd's sample of the jump times, a level per segment."""
    key = _mix((seed + 0x9E3779B97F4A7C15 * (k + 1)) & _M64)
    N, S = nt - 1, set()
    for q, j in enumerate(range(N - jumps + 1, N + 1)):
        t = 1 + _uniform(key, 1, q, j)
        S.add(j if t in S else t)
    u = np.zeros((levels.M, nt))
    seg = 0
    for i in range(nt):
        seg += i in S
        u[:, i] = levels.nuval[_uniform(key, 2, seg, levels.L)]
    return u, S


@pytest.mark.parametrize("shape", ["sos1", "c5", "c4"])
def test_rand_start_device(shape):
    """Admissible piecewise-constant starts with exactly `jumps` distinct candidate jump times in 1..nt-1; the
    device stream equals its host restatement bit for bit; seeds reproduce; jump times are uniform over steps."""
    import torch
    from mioc.synth import CONFIGS
    lt = {"sos1": LevelTable([[0, 1]] * 3, mioc.bounded_sum_iterator([[0, 1]] * 3, 1, 1)),
          "c5": CONFIGS["C5"].levels(), "c4": CONFIGS["C4"].levels()}[shape]
    nt = {"sos1": 512, "c5": 4096, "c4": 65536}[shape]
    K = {"sos1": 256, "c5": 64, "c4": 4}[shape]
    ctx = native.Context(0)
    ctx.set_levels(lt)
    out = torch.empty(K, nt, lt.M, dtype=torch.float64, device="cuda")
    ctx.rand_start_tensor(out, seed=1234)
    out2 = torch.empty_like(out)
    ctx.rand_start_tensor(out2, seed=1234)
    out3 = torch.empty_like(out)
    ctx.rand_start_tensor(out3, seed=1235)
    ctx.synchronize()
    u = out.cpu().numpy()
    assert torch.equal(out, out2) and not torch.equal(out, out3)
    rows = {tuple(r) for r in lt.nuval}
    jumps = nt // 10
    hits = np.zeros(nt)
    for k in range(K):
        assert all(tuple(c) in rows for c in u[k])
        changes = np.flatnonzero(np.any(u[k][1:] != u[k][:-1], axis=1)) + 1
        assert changes.size <= jumps
        if k < 3:
            hu, S = _rand_start_host(lt, nt, jumps, 1234, k)
            assert np.array_equal(u[k].T, hu) and len(S) == jumps and set(changes) <= S
        hits[changes] += 1
    if shape == "sos1":  # each step 1..nt-1 is a candidate with probability jumps/(nt-1); a change needs a new level
        p = jumps / (nt - 1) * (2 / 3)
        assert abs(hits[1:].mean() / K - p) < 0.1 * p
    with pytest.raises(native.MiocNativeError):
        ctx.rand_start_tensor(out, seed=1, jumps=nt)
    ctx.close()


class _DeviceODE:
    """Test double: an ODE example whose eval_f! / eval_df! run through mioc_ode_eval_device for one restart, so
    the host TRM (multi-trust.jl mirror) and TRM_batch see bit-identical objective values and gradients."""

    def __new__(cls, name, nt, ctx):
        import torch
        obj = _obj(name, nt)
        prob = dict((c[0], c[1]) for c in CASES)[name]

        def f_helper(x, cache):
            X = torch.tensor(np.ascontiguousarray(np.asarray(x).T[None]), dtype=torch.float64, device="cuda")
            J = torch.empty(1, dtype=torch.float64, device="cuda")
            ctx.ode_eval_tensors(prob, X, obj.T0, obj.T1, J, None)
            ctx.synchronize()
            return J.item()

        def df_helper():
            X = torch.tensor(np.ascontiguousarray(obj.x.T[None]), dtype=torch.float64, device="cuda")
            D = torch.empty_like(X)
            ctx.ode_eval_tensors(prob, X, obj.T0, obj.T1, None, D)
            ctx.synchronize()
            obj.df[:, :] = D[0].cpu().numpy().T

        obj.eval_f_helper = f_helper
        obj.eval_df_helper = df_helper
        return obj


@pytest.mark.parametrize("name,p,nt", [("fishing", math.inf, 240), ("doubletank", math.inf, 240),
                                       ("vanderpol", 1, 2000)])
def test_trm_batch_equals_sequential_trm(name, p, nt):
    """TRM_batch (every restart's data on the device, decisions per inner iteration) against the host TRM loop
    (multi-trust.jl:53-170 mirror) run restart by restart with the same device kernels: identical returned values
    J + β·TV_p(u) and identical controls obj.x, including restarts that halve Δ and that stop on pred <= 0."""
    import torch
    from mioc.trm_batch import TRM_batch
    K = 12  # vanderpol: explicit Euler needs the example's own nt = 2000 over T = 20 to stay finite
    par = mioc.TRM_parameters(beta=1e-3, Delta0=1.0, p=p, maxiter=6, kmax=5)
    ctx = native.Context(0)
    ctx.set_levels(LevelTable([[0, 1]] * 3, mioc.bounded_sum_iterator([[0, 1]] * 3, 1, 1)))
    x0 = torch.empty(K, nt, 3, dtype=torch.float64, device="cuda")
    ctx.rand_start_tensor(x0, seed=99)
    ctx.synchronize()
    log = []
    vals, u, iters = TRM_batch(name, par, x0=x0, log=log)
    ub = u.cpu().numpy()
    halvings = sum(int(np.sum(d == 1)) for *_, d, _inner in log)
    for k in range(K):
        obj = _DeviceODE(name, nt, ctx)
        J = mioc.TRM(obj, par, x0=x0[k].cpu().numpy().T.copy())
        assert J == vals[k], (k, J, vals[k])
        assert np.array_equal(obj.x, ub[k].T), k
    print(f"{name}: iterations per restart {iters.tolist()}, halvings {halvings}")
    ctx.close()


@pytest.mark.parametrize("chunk", [1, 2, 3])
def test_trm_batch_production_path_equals_logged_and_sequential(chunk):
    """The production path of TRM_batch (log=None: no decision array, several trials enqueued between two read-backs
    of the control flags, gated kernels skipped by restarts that left their inner loop) against the logged path
    (one synchronisation per trial) and against the host TRM loop run restart by restart: identical values,
    controls and iteration counts.  kmax = 3 with chunks of 1, 2 and 3 trials: an inner loop ends at every position
    of a chunk (mid-chunk for chunk 2, at a chunk end for 1 and 3)."""
    import torch
    from mioc.trm_batch import TRM_batch
    K, nt = 12, 240
    par = mioc.TRM_parameters(beta=1e-3, Delta0=1.0, p=math.inf, maxiter=6, kmax=3)
    ctx = native.Context(0)
    ctx.set_levels(LevelTable([[0, 1]] * 3, mioc.bounded_sum_iterator([[0, 1]] * 3, 1, 1)))
    x0 = torch.empty(K, nt, 3, dtype=torch.float64, device="cuda")
    # the first of a few fixed (problem, seed) whose starts make some restart halve its radius (an inner loop of
    # length > 1)
    for name, seed in [(nm, sd) for nm in ("doubletank", "fishing") for sd in (1234, 99, 7, 2024)]:
        ctx.rand_start_tensor(x0, seed=seed)
        ctx.synchronize()
        log = []
        vl, ul, il = TRM_batch(name, par, x0=x0, log=log)
        halvings = sum(int(np.sum(d == 1)) for *_, d, _inner in log)
        if halvings >= 1:
            break
    assert halvings >= 1, "no restart halved its radius: the chunked inner loop was not exercised"
    print(f"{name} seed {seed}: halvings {halvings}")
    stats = {}
    vals, u, iters = TRM_batch(name, par, x0=x0, inner_chunk=chunk, stats=stats)
    assert np.array_equal(vals, vl) and np.array_equal(iters, il)
    assert torch.equal(u, ul)
    assert stats["polls"] <= stats["outer"] * -(-par.kmax // chunk)
    ub = u.cpu().numpy()
    for k in range(K):
        obj = _DeviceODE(name, nt, ctx)
        J = mioc.TRM(obj, par, x0=x0[k].cpu().numpy().T.copy())
        assert J == vals[k], (k, J, vals[k])
        assert np.array_equal(obj.x, ub[k].T), k
    ctx.close()
