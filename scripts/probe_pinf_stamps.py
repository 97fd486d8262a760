"""Phase cycles of k_pinf_recur per step (diagnostic build libmioc_stamps.so, s_memtime, workgroup 0)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", "libmioc_stamps.so")
sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
import numpy as np
from mioc import native
from mioc.synth import CONFIGS, make_inputs
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cfg = CONFIGS["C4"]
lt, df, uo = make_inputs(cfg, nt=nt)
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(float("inf"), cfg.beta)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
ctx.bellman(df, uo, cfg.B, cfg.dt); ctx.synchronize()
ms, n, name = ctx.kernel_stats(0)
print(f"{name}: {ms:.2f} ms for nt={nt} ({1e6 * ms / 1e3 / max(nt - 1, 1):.0f} ns/step)")
buf = (ctypes.c_ulonglong * (16 * 8))()
lib = native.load_library()
f = lib.mioc_debug_pinf_stamps; f.argtypes = [ctypes.c_void_p]; f.restype = ctypes.c_int32
assert f(buf) == 0
st = np.array(buf, dtype=np.int64).reshape(16, 8)
for w in range(16):
    if st[w, 3] == 0:
        continue
    n = st[w, 3]
    print(f"wave {w}: steps {n}  cycles/step: reads waited {st[w,0]/n:7.0f}  VALU+stores {(st[w,1]-st[w,0])/n:7.0f}"
          f"  barrier {st[w,2]/n:7.0f}  total {st[w,4]/n:7.0f}")
# backtrack walk: walker (wave 0 of workgroup 0) cycles per step, and the chunk-end wait (staging not landed)
ctx.set_option(native.MIOC_OPT_TIMING, 1)
ctx.reset_stats()
ctx.backtrack(cfg.B)
ms, n, name = ctx.kernel_stats(1)
assert f(buf) == 0
st = np.array(buf, dtype=np.int64).reshape(16, 8)
steps, chunks = max(st[8, 3], 1), max(st[8, 2], 1)
print(f"{name}: {ms:.2f} ms; walker cycles/step {st[8,0]/steps:.0f} (incl. staging issue), chunk-end wait "
      f"{st[8,1]/chunks:.0f} cycles/chunk over {chunks} chunks of {steps/chunks:.1f} steps")
