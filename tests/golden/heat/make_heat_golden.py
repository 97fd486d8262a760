"""Generate the heat fixture tests/golden/heat/heat_n5_nt24.npz from the CPU oracle (oracle/heat_oracle.py, the LU
restatement of julia_opt/PDEObjective.jl:129-199).  Run:  python tests/golden/heat/make_heat_golden.py
The reference (Julia + its FEM bundle) cannot run here and holds no heat outputs, so this fixture anchors the
oracle and the device against a committed vector, not against Julia.  Arrays only (allow_pickle=False):
  M_invA, M_invF, M, state0, yd (the stand-in P1 problem, mioc/heat.py, n = 5 -> N = 25), scalars [T0, T1, gamma],
  x (K x nx x nt controls), J (K), df (K x nx x nt)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")]

from mioc.heat import HeatProblem  # noqa: E402
from oracle.heat_oracle import HeatOracle  # noqa: E402

hp = HeatProblem(n=5, nt=24)
o = HeatOracle(hp.M_invA, hp.M_invF, hp.M, hp.state0, hp.yd, hp.T0, hp.T1, hp.gamma)
rng = np.random.default_rng(2024)
xs = np.stack([rng.integers(0, 6, size=(2, hp.nt)).astype(np.float64) for _ in range(4)])
res = [o.eval(x)[:2] for x in xs]
np.savez(os.path.join(HERE, "heat_n5_nt24.npz"), M_invA=hp.M_invA, M_invF=hp.M_invF, M=hp.M, state0=hp.state0,
         yd=hp.yd, scalars=np.array([hp.T0, hp.T1, hp.gamma]), x=xs, J=np.array([r[0] for r in res]),
         df=np.stack([r[1] for r in res]))
print("wrote heat_n5_nt24.npz")
