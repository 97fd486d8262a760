import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libmioc.so)")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    d = {k: z[k] for k in z.files}
    B, Bp, beta, dt, pk, pint = d["scalars"]
    d.update(B=int(B), Bp=int(Bp), beta=float(beta), dt=float(dt), p_kind=int(pk), p_int=int(pint))
    counts = d["nu_counts"]
    vals = d["nu_values"]
    nu, o = [], 0
    for c in counts:
        nu.append([int(x) for x in vals[o:o + c]])
        o += c
    d["nu"] = nu
    d["tuple_list"] = [tuple(int(x) for x in t) for t in d["tuples"]]
    d["name"] = os.path.splitext(os.path.basename(path))[0]
    return d


@pytest.fixture(scope="session")
def oracle_c():
    from oracle.oracle import OracleC
    return OracleC()
