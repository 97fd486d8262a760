"""Phase timing of the separable-transform kernel (diagnostic build libmioc_stamps.so, s_memtime per workgroup;
s_memrealtime for the launch timeline)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", "libmioc_stamps.so")
sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 64
persist = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_SEPARABLE)
ctx.set_option(native.MIOC_OPT_PERSIST, persist)
ctx.bellman(df, uo, cfg.B, cfg.dt)  # warm-up
ctx.synchronize()
ctx.bellman(df, uo, cfg.B, cfg.dt)
ctx.synchronize()
print("persistent" if persist else "per-step launches")
nb = cfg.B + 1
buf = (ctypes.c_ulonglong * (nb * 16))()
lib = native.load_library()
f = lib.mioc_debug_sdt_stamps; f.argtypes = [ctypes.c_void_p, ctypes.c_int64]; f.restype = ctypes.c_int32
assert f(buf, nb) == 0
st = np.array(buf, dtype=np.int64).reshape(nb, 16)
seq = [(0, "start"), (1, "loads+reduce+barrier"), (2, "stamp+barrier"), (3, "pass 0"), (4, "pass 1"),
       (5, "pass 2"), (6, "pass 3"), (7, "targets+list+barrier"), (8, "exact scans"), (9, "Sout gather+store")]
full = st[:, 9] > 0
print("blocks with all stamps:", full.sum(), "of", nb)
s = st[full & (st[:, 6] > 0)]
for (a, _), (b, nm) in zip(seq[:-1], seq[1:]):
    d = s[:, b] - s[:, a]
    print(f"{nm:22s} cycles median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}  max {d.max():9.0f}")
tot = s[:, 9] - s[:, 0]
print(f"{'total':22s} cycles median {np.median(tot):9.0f}  max {tot.max():9.0f}")
rt0, rt1 = st[:, 13], st[:, 14]
ok = (rt0 > 0) & (rt1 > 0)
t0 = rt0[ok].min()
s_us, e_us = (rt0[ok] - t0) / 100.0, (rt1[ok] - t0) / 100.0
print(f"realtime: kernel span {e_us.max():.2f} us; start spread p50/p90/p99/max {np.percentile(s_us, [50, 90, 99, 100])} us;"
      f" end median {np.median(e_us):.2f} p90 {np.percentile(e_us, 90):.2f} max {e_us.max():.2f} us")
order = np.argsort(s_us)
idx = np.nonzero(ok)[0]
print("latest starters (row, start us, dur us):", [(int(idx[i]), round(float(s_us[i]), 2),
      round(float(e_us[i] - s_us[i]), 2)) for i in order[-4:]])
print("longest rows (row, dur us):", sorted([(int(idx[i]), round(float(e_us[i] - s_us[i]), 2))
      for i in range(len(s_us))], key=lambda t: -t[1])[:6])
ms, n, name = ctx.kernel_stats(0)
print("diagnostics", ctx.diagnostics())
