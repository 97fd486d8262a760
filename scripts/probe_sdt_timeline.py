"""Timeline of the pipelined persistent separable-transform kernel (diagnostic build libmioc_stamps_tl.so, `make
stamps_tl`): for every row and the 64 steps from nt/2 down, s_memrealtime (100 MHz) at 8 points of the row body:
0 start, 7 loads taken, 1 dependency polls issued (after the first barrier), 2 go()
(the first barrier passed), 3 polls matched, 4 next row's loads and copies issued, 5 previous row's stores drained (late,
before the winners' barrier), 6 stores issued.  Prints the phase durations, the step period and the pipeline skew between neighbouring rows.
Usage: python scripts/probe_sdt_timeline.py [nt] [NB]  [save.npy] [--lib another timeline build]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
_lib = os.path.join(PKG, "lib", "libmioc_stamps_tl.so")
if "--lib" in sys.argv:  # another timeline build (e.g. make variant VFLAGS="-DMIOC_STAMPS -DMIOC_STAMPS_TL ...")
    q = sys.argv.index("--lib")
    _lib = sys.argv[q + 1]
    del sys.argv[q:q + 2]
os.environ["MIOC_LIB"] = _lib
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
with native.Context(0) as ctx:
    ctx.set_levels(lt)
    ctx.set_cost(1, cfg.beta)
    ctx.set_option(native.MIOC_OPT_ALGO, native.MIOC_ALGO_SEPARABLE)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)
    ctx.set_option(native.MIOC_OPT_PERSIST, 1)
    ctx.set_option(native.MIOC_OPT_SDT_BUFFERS, nb)
    ctx.bellman(df, uo, cfg.B, cfg.dt)  # warm-up: code object load, first touch of the buffers
    ctx.synchronize()
    ctx.reset_stats()
    ctx.bellman(df, uo, cfg.B, cfg.dt)
    ctx.synchronize()
    ms, n, name = ctx.kernel_stats(0)
    print(f"{name}: {ms:.3f} ms for {nt - 1} steps = {1e3 * ms / (nt - 1):.3f} us/step (NB={nb}); "
          f"diagnostics {ctx.diagnostics()}")
    R = cfg.B + 1
    lib = native.load_library()
    f = lib.mioc_debug_sdt_timeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    f.restype = ctypes.c_int32
    buf = (ctypes.c_ulonglong * (R * 64 * 8))()
    assert f(buf, R) == 0
tl = np.array(buf, dtype=np.int64).reshape(R, 64, 8).astype(np.float64) / 100.0  # us
if len(sys.argv) > 3:
    np.save(sys.argv[3], tl)
rows = np.arange(1, R)  # row 0 has no workgroup
steps = np.arange(2, 62)
T = tl[rows][:, steps, :]
ok = np.all(T[:, :, :8] > 0, axis=2)
names = ["row start -> polls issued (0->1)", "polls issued -> go (1->2)", "poll wait at go (2->3)",
         "issue next loads + copies (3->4)", "-> late drain done (4->5)", "list barrier, scans, stores (5->6)"]
for q, nm in enumerate(names):
    d = (T[:, :, q + 1] - T[:, :, q])[ok]
    print(f"{nm:36s} median {np.median(d):6.3f}  p10 {np.percentile(d, 10):6.3f}  p90 {np.percentile(d, 90):6.3f} us")
# period: start of step i-1 minus start of step i, same row (steps descend with the index here)
per = (T[:, 1:, 0] - T[:, :-1, 0])
print(f"step period per row: median {np.median(per):.3f}  p10 {np.percentile(per, 10):.3f}  p90 "
      f"{np.percentile(per, 90):.3f} us")
if os.environ.get("TL_DRAIN"):  # a -DSD_TL_DRAIN build: stamp 7 is the late drain's start
    for nm, a, b in (("  passes + winners (4->7)", 4, 7), ("  late drain wait (7->5)", 7, 5)):
        d = (T[:, :, b] - T[:, :, a])[ok]
        print(f"{nm:36s} median {np.median(d):6.3f}  p10 {np.percentile(d, 10):6.3f}  p90 {np.percentile(d, 90):6.3f} us")
d = (T[:, :, 7] - T[:, :, 0])[ok]
print(f"{'  of it: waiting for the loads (0->7)':36s} median {np.median(d):6.3f}  p10 {np.percentile(d, 10):6.3f}  p90 {np.percentile(d, 90):6.3f} us")
rest = (T[:, 1:, 0] - T[:, :-1, 6])
print(f"stores issued -> next row start: median {np.median(rest):.3f} us")
skew = T[1:, :, 0] - T[:-1, :, 0]  # row c starts step i this long after row c-1
print(f"skew row c vs row c-1 (same step start): median {np.median(skew):.3f}  p10 {np.percentile(skew, 10):.3f}  "
      f"p90 {np.percentile(skew, 90):.3f} us; total over rows 1..{R - 1}: {np.median(T[-1, :, 0] - T[0, :, 0]):.1f} us")
by_row = np.median(T[:, :, 3] - T[:, :, 2], axis=1)
print("poll wait by row (median, every 16th row):", [round(float(x), 3) for x in by_row[::16]])
ld = np.median(T[:, :, 7] - T[:, :, 0], axis=1)
print("load wait by row (median, every 16th row):", [round(float(x), 3) for x in ld[::16]])
