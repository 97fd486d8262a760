"""Persistent separable-transform kernel timeline (diagnostic build libmioc_stamps_tl.so, make stamps_tl): per row and step
(i < 64) the dependency-wait begin/end, row-body end and done publish (s_memrealtime, 100 MHz), plus the
in-row phase clocks of the last processed row (s_memtime)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", "libmioc_stamps_tl.so")
sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_SEPARABLE)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
ctx.set_option(native.MIOC_OPT_PERSIST, 1)
ctx.bellman(df, uo, cfg.B, cfg.dt)  # warm-up: code object load, first-touch of the buffers
ctx.synchronize()
ctx.reset_stats()
ctx.bellman(df, uo, cfg.B, cfg.dt)
ctx.synchronize()
ms, n, name = ctx.kernel_stats(0)
print(f"{name}: {ms:.3f} ms for {nt - 1} steps = {1e3 * ms / (nt - 1):.2f} us/step")
nb = cfg.B + 1
lib = native.load_library()
f = lib.mioc_debug_sdt_timeline; f.argtypes = [ctypes.c_void_p, ctypes.c_int64]; f.restype = ctypes.c_int32
buf = (ctypes.c_ulonglong * (nb * 64 * 4))()
assert f(buf, nb) == 0
tl = np.array(buf, dtype=np.int64).reshape(nb, 64, 4)
steps = range(2, 62)
t0 = tl[:, 2:62, :][tl[:, 2:62, :] > 0].min()
W = (tl[:, steps, 1] - tl[:, steps, 0]) / 100.0   # us waiting
Bd = (tl[:, steps, 2] - tl[:, steps, 1]) / 100.0  # us row body
Pu = (tl[:, steps, 3] - tl[:, steps, 2]) / 100.0  # us drain + publish
print("per row-step (us): wait median %.2f p90 %.2f | body median %.2f p90 %.2f max %.2f | drain+publish median %.2f p90 %.2f"
      % (np.median(W), np.percentile(W, 90), np.median(Bd), np.percentile(Bd, 90), Bd.max(), np.median(Pu), np.percentile(Pu, 90)))
# step period: time between consecutive done publishes of the same row
per = -np.diff(tl[:, steps, 3], axis=1) / 100.0
print("step period per row (us): median %.2f p10 %.2f p90 %.2f" % (np.median(per), np.percentile(per, 10), np.percentile(per, 90)))
# critical chain: done(row) at step i vs the latest done among its sources at step i+1
lag = []
for i in range(2, 61):
    for c in range(nb):
        src = tl[max(0, c - 28):c + 1, i + 1, 3]
        lag.append((tl[c, i, 1] - src.max()) / 100.0)
lag = np.array(lag)
print("hand-off latency (latest source done -> wait end) us: median %.2f p90 %.2f" % (np.median(lag), np.percentile(lag, 90)))
body_by_row = np.median(Bd, axis=1)
print("slowest rows by median body (row, us):", sorted([(int(r), round(float(body_by_row[r]), 2)) for r in range(nb)], key=lambda t: -t[1])[:6])
print("diagnostics", ctx.diagnostics())
# which dependency gates each row: RAW (rows c'-28..c'-1 of step i+1 done) vs WAR (rows c'+1..c'+28 of
# step i+2 past their loads; approximated by their wait end + 3 us) vs the workgroup's own previous row
raw_gap, war_gap, by_row = [], [], np.zeros(nb)
for c in range(nb):
    g = []
    for i in range(2, 60):
        raw = tl[max(0, c - 28):c, i + 1, 3].max() if c > 0 else 0
        war = tl[c + 1:c + 29, i + 2, 1].max() if c + 1 < nb else 0
        g.append((tl[c, i, 1] - raw) / 100.0)
        war_gap.append((tl[c, i, 1] - war) / 100.0)
    by_row[c] = np.median(g)
    raw_gap += g
raw_gap, war_gap = np.array(raw_gap), np.array(war_gap)
print("wait end - latest RAW done (us): median %.2f p10 %.2f p90 %.2f" % (np.median(raw_gap), np.percentile(raw_gap, 10), np.percentile(raw_gap, 90)))
print("wait end - latest WAR wait end at i+2 (us): median %.2f p10 %.2f p90 %.2f" % (np.median(war_gap), np.percentile(war_gap, 10), np.percentile(war_gap, 90)))
print("median (wait end - RAW done) by row, every 8th row:", [round(float(x), 2) for x in by_row[::8]])
st = tl[:, 10, 1] / 100.0
print("step 10 wait end relative to row 0 (us), every 8th row:", [round(float(x), 2) for x in (st - st[0])[::8]])
ref = tl[0, 14, 0]
for c in (0, 1, 2, 28, 29, 128, 227, 228, 255, 256):
    print(f"row {c:3d} steps 14..10 [wait begin, wait end, body end, done] us rel.:",
          [[round((int(x) - int(ref)) / 100.0, 2) for x in tl[c, i]] for i in range(14, 9, -1)])
