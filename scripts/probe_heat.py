"""A/B timing of k_heat_run builds: MIOC_LIB=<lib> python scripts/probe_heat.py [K] [n] [nt].
Times one eval_f + eval_df launch for K restarts (HIP events on the library's stream, 5 launches) and checks two
restarts against the LU oracle."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mioc import native  # noqa: E402
from mioc.heat import HeatProblem  # noqa: E402
from oracle.heat_oracle import HeatOracle  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = int(sys.argv[2]) if len(sys.argv) > 2 else 17
nt = int(sys.argv[3]) if len(sys.argv) > 3 else 500
hp = HeatProblem(n=n, nt=nt)
ctx = native.Context(0)
hp.setup(ctx)
g = torch.Generator().manual_seed(5)
x = torch.randint(0, 6, (K, nt, 2), generator=g).double().cuda()
J = torch.empty(K, dtype=torch.float64, device="cuda")
df = torch.empty_like(x)
st = torch.cuda.ExternalStream(ctx.stream())
ctx.heat_eval_tensors(x, J, df)
ctx.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(st)
for _ in range(5):
    ctx.heat_eval_tensors(x, J, df)
ev[1].record(st)
ctx.synchronize()
ms = ev[0].elapsed_time(ev[1]) / 5
o = HeatOracle(hp.M_invA, hp.M_invF, hp.M, hp.state0, hp.yd, hp.T0, hp.T1, hp.gamma)
ok = True
for k in (0, K - 1):
    fo, dfo, _ = o.eval(x[k].cpu().numpy().T)
    ok &= abs(J[k].item() - fo) <= 1e-9 * abs(fo)
    ok &= np.max(np.abs(df[k].cpu().numpy().T - dfo)) <= 1e-9 * np.max(np.abs(dfo))
N = hp.N
tf = 6.0 * N * N * nt * K / (ms / 1e3) / 1e12
print(f"{os.path.basename(os.environ.get('MIOC_LIB', 'libmioc.so'))}: K={K} N={N} nt={nt} {ms:.3f} ms/launch "
      f"{tf:.2f} TFLOP/s parity={'ok' if ok else 'FAIL'} J0={J[0].item():.17g}", flush=True)
ctx.close()
