"""Wall time of the multi-start TRM on the heat example entirely on the device (mioc.trm_batch.TRM_batch with a
HeatProblem): python scripts/probe_heat_trm.py [K] [n] [nt] [maxiter]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mioc  # noqa: E402
from mioc.heat import HeatProblem  # noqa: E402
from mioc.trm_batch import TRM_batch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 17
nt = int(sys.argv[3]) if len(sys.argv) > 3 else 500
maxiter = int(sys.argv[4]) if len(sys.argv) > 4 else 10
hp = HeatProblem(n=n, nt=nt)
par = mioc.TRM_parameters(beta=1e-2, Delta0=2.0, p=1, maxiter=maxiter, kmax=10)
TRM_batch(hp, par, K=16, seed=1)  # warm-up (setup, code objects)
torch.cuda.synchronize()
t0 = time.perf_counter()
stats = {}
vals, u, iters = TRM_batch(hp, par, K=K, seed=2, stats=stats)  # the product path: no per-trial log
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"heat TRM_batch: K={K} N={hp.N} nt={nt} maxiter={maxiter}: {dt:.3f} s = {K / dt:.1f} restarts/s; "
      f"outer iterations {stats['outer']} (per restart mean {iters.mean():.2f}); host read-backs of the control "
      f"flags {stats['polls']} = {stats['polls'] / max(1, stats['outer']):.2f} per outer iteration; "
      f"J+beta*TV min {np.min(vals):.6g} median {np.median(vals):.6g}", flush=True)
log = []
vals2, _, iters2 = TRM_batch(hp, par, K=K, seed=2, log=log)  # the same run with a per-trial log (debugging)
print(f"  with the per-trial log: {len(log)} inner iterations, same values: {bool(np.array_equal(vals, vals2))}, "
      f"same iterations: {bool(np.array_equal(iters, iters2))}", flush=True)
