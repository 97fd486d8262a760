"""Phase timing of the pyramid kernel (diagnostic build libmioc_stamps.so, s_memtime per workgroup)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", "libmioc_stamps.so")
sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 64
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta); ctx.set_option(native.MIOC_OPT_ALGO, 3)
ctx.bellman(df, uo, cfg.B, cfg.dt)
nb = cfg.B + 1
buf = (ctypes.c_ulonglong * (nb * 16))()
lib = native.load_library()
f = lib.mioc_debug_pyr_stamps; f.argtypes = [ctypes.c_void_p, ctypes.c_int64]; f.restype = ctypes.c_int32
assert f(buf, nb) == 0
st = np.array(buf, dtype=np.int64).reshape(nb, 16)
# stamp slots in program order (6 holds the number of levels)
seq = [(0, "start"), (1, "load+T1+reduce"), (2, "delta+fq+clears"), (7, "barrier"), (8, "inserts"),
       (9, "barrier"), (3, "border marks"), (4, "pyramid"), (10, "lookups"), (11, "outnat+UU+barrier"),
       (12, "Sout gather+store"), (5, "exact scans")]
full = st[:, 5] > 0
print("blocks with all stamps:", full.sum(), "of", nb)
s = st[full]
for (a, _), (b, nm) in zip(seq[:-1], seq[1:]):
    d = s[:, b] - s[:, a]
    print(f"{nm:22s} cycles median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}  max {d.max():9.0f}")
tot = s[:, 5] - s[:, 0]
print(f"{'total':22s} cycles median {np.median(tot):9.0f}  max {tot.max():9.0f}")
print("levels executed: median", np.median(s[:, 6]), "max", s[:, 6].max(), "min", s[:, 6].min())
# global timeline (s_memrealtime, 100 MHz): when each workgroup started / ended relative to the first start
rt0, rt1 = st[:, 13], st[:, 14]
ok = (rt0 > 0) & (rt1 > 0)
t0 = rt0[ok].min()
s_us, e_us = (rt0[ok] - t0) / 100.0, (rt1[ok] - t0) / 100.0
print(f"realtime: kernel span {e_us.max():.1f} us; start spread {np.percentile(s_us, [50, 90, 99, 100])} us;"
      f" end median {np.median(e_us):.1f} p90 {np.percentile(e_us, 90):.1f} max {e_us.max():.1f} us")
order = np.argsort(s_us)
print("latest starters (row, start us, dur us):", [(int(np.nonzero(ok)[0][i]), round(float(s_us[i]), 1),
      round(float(e_us[i] - s_us[i]), 1)) for i in order[-3:]])
print("longest rows (row, dur us):", sorted([(int(np.nonzero(ok)[0][i]), round(float(e_us[i] - s_us[i]), 1))
      for i in range(len(s_us))], key=lambda t: -t[1])[:5])
dl = st[full, 15]
tot_wl, chg_wl = dl >> 32, dl & 0xFFFFFFFF
print(f"wave-levels with a BM change: {chg_wl.sum()} of {tot_wl.sum()} ({100.0 * chg_wl.sum() / max(1, tot_wl.sum()):.1f}%)")
