"""CPU tier: the ODE gradient oracle (oracle/ode_oracle.py, restating ODEObjective.jl:125-184 with the hooks of
example_fishing.jl / example_doubletank.jl / example_vanderpol.jl) pinned the way the reference pins its own gradients
(test_df, example_fishing.jl:94-123): finite differences of eval_f against tau * sum_i df_i' h_i; and agreement with
the product's independent host mirror (mioc/ode.py) to rounding."""
import random

import numpy as np
import pytest

from oracle.ode_oracle import ODEOracle

CASES = [("fishing", 240), ("doubletank", 200), ("vanderpol", 2000)]


def _x(nt, seed, sos1=True):
    rnd = random.Random(seed)
    if sos1:  # admissible SOS1 controls (bounded_sum_iterator(V, 1, 1))
        return [tuple(1.0 if m == rnd.randrange(3) else 0.0 for m in range(3)) for _ in range(nt)]
    return [tuple(0.5 for _ in range(3)) for _ in range(nt)]  # test_df's x .= .5


@pytest.mark.parametrize("name,nt", CASES, ids=[c[0] for c in CASES])
def test_ode_oracle_finite_differences(name, nt):
    o = ODEOracle(name, nt)
    rnd = random.Random(7)
    x = _x(nt, 3, sos1=False)
    h = [tuple(rnd.gauss(0, 1) for _ in range(3)) for _ in range(nt)]
    errs = [o.fd_check(x, h, t) for t in (1e-4, 1e-5, 1e-6)]
    scale = max(1e-12, errs[0][1])
    # first-order FD: the error falls with t until rounding takes over; at 1e-6 it is tiny against |dfh|
    assert errs[2][0] <= 1e-4 * scale + 1e-9, errs
    assert errs[1][0] <= errs[0][0] * 0.5 + 1e-9, errs


@pytest.mark.parametrize("name,nt", CASES, ids=[c[0] for c in CASES])
def test_ode_oracle_matches_host_mirror(name, nt):
    import mioc
    from mioc.ode import DTMObj, LVMObj, VPOObj
    obj = {"fishing": LVMObj, "doubletank": DTMObj, "vanderpol": VPOObj}[name](nt=nt)
    o = ODEOracle(name, nt)
    assert o.tau == obj.tau and o.state0 == tuple(obj.state0)
    for seed in range(3):
        x = _x(nt, seed)
        J, df = o.eval_df(x)
        obj.x[:, :] = np.array(x).T
        Jm = mioc.eval_f_(obj)
        mioc.eval_df_(obj)
        assert abs(J - Jm) <= 1e-12 * abs(J), (J, Jm)
        d = np.array(df).T
        assert np.max(np.abs(d - obj.df)) <= 1e-12 * np.max(np.abs(d)), seed
