"""Phase clocks of the round-3 fused separable DP (diagnostic build libmioc_stamps.so, `make stamps`): per wave,
s_memtime cycles summed over the steps at 8 points of a step, printed as cycles per step (mean over waves):
0 read + statistics + stamps, 1 passes, 2 winners, 3 exact scans + the extra row, 4 drain + barrier 1,
5 write phase, 6 barrier 2, 7 the whole step.  Usage: python scripts/probe_fsep_phases.py K S [nt]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", os.environ.get("FS_LIB", "libmioc_stamps.so"))
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 16
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nt = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
cfg = CONFIGS["C5"]
lt = cfg.levels()
dfs, uos = [], []
for k in range(K):
    _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=lt)
    dfs.append(df)
    uos.append(uo)
ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64, device="cuda")
duo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64, device="cuda")
with native.Context(0) as ctx:
    ctx.set_levels(lt)
    ctx.set_cost(cfg.p, cfg.beta)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_FUSED_SEPARABLE)
    ctx.set_option(native.MIOC_OPT_FSEP_SEGMENTS, S)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    ctx.synchronize()
    ctx.reset_stats()
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    ctx.synchronize()
    ms, n, name = ctx.kernel_stats(0)
    d = ctx.diagnostics()
    lib = native.load_library()
    f = lib.mioc_debug_fsep_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    f.restype = ctypes.c_int32
    nw = min(4096, K * d[8] * 8)
    buf = (ctypes.c_ulonglong * (nw * 8))()
    assert f(buf, nw) == 0
a = np.array(buf, dtype=np.float64).reshape(nw, 8) / (nt - 1)
wpb = int(os.environ.get("FS_WPB", 8 if d[8] <= 1 else max(1, 8 // d[8])))  # waves per workgroup (B = 256; FS_WPB: four lanes per row)
per_wave = a[: (len(a) // wpb) * wpb].reshape(-1, wpb, 8)
a = a[a[:, 7] > 0]
us = 1e3 * ms / (nt - 1)
print(f"{name} K={K} S={d[8]} nt={nt}: {us:.3f} us/step; waves sampled {len(a)}")
names = ["read+stats+stamp", "passes", "winners", "scans+extra", "drain+barrier1", "write phase", "barrier2", "step"]
for q, nm in enumerate(names):
    print(f"  {nm:18s} mean {a[:, q].mean():8.0f}  min {a[:, q].min():8.0f}  max {a[:, q].max():8.0f} cycles/step"
          f"   by wave: {[int(x) for x in per_wave[:, :, q].mean(axis=0)]}")
