"""C5 batch through the fused small-state DP: kernel time (HIP events) and, with the diagnostic build
(argv[2] == 'stamps': libmioc_stamps.so), cycles per step and phase summed over the launch per workgroup."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
stamps = len(sys.argv) > 2 and sys.argv[2] == "stamps"
if stamps:
    os.environ["MIOC_LIB"] = os.path.join(PKG, "lib", "libmioc_stamps.so")
sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
import numpy as np
import torch
from mioc import native
from mioc.synth import CONFIGS, make_inputs
K = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
algo = int(sys.argv[3]) if len(sys.argv) > 3 else native.MIOC_ALGO_FUSED
cfg = CONFIGS["C5"]
lt = cfg.levels()
dfs, uos = [], []
for k in range(K):
    _, df, uo = make_inputs(cfg, k=k, levels=lt)
    dfs.append(df.T); uos.append(uo.T)
ddf = torch.tensor(np.ascontiguousarray(np.stack(dfs)), dtype=torch.float64, device="cuda")
duo = torch.tensor(np.ascontiguousarray(np.stack(uos)), dtype=torch.float64, device="cuda")
ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
ctx.set_option(native.MIOC_OPT_ALGO, algo); ctx.set_option(native.MIOC_OPT_TIMING, 1)
for rep in range(3):
    ctx.reset_stats()
    ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
    ctx.synchronize()
    ms, n, name = ctx.kernel_stats(0)
    print(f"{name}: {ms:.3f} ms for K={K}  -> {K / ms * 1e3:.1f} subproblems/s, {ms * 1e3 / (cfg.nt - 1):.2f} us per DP step")
print("diagnostics", ctx.diagnostics())
if stamps:
    lib = native.load_library()
    f = lib.mioc_debug_fused_stamps; f.argtypes = [ctypes.c_void_p, ctypes.c_int64]; f.restype = ctypes.c_int32
    nb = 4096
    buf = (ctypes.c_ulonglong * (nb * 8))()
    assert f(buf, nb) == 0
    st = np.array(buf, dtype=np.int64).reshape(nb, 8) / (cfg.nt - 1)
    names = (["tasks (compute + U stores)", "prepare next step", "barrier A wait", "front writes", "barrier B wait"]
             if algo == native.MIOC_ALGO_FUSED else
             ["load + stats + stamp", "transform", "targets", "exact scans", "barrier A wait", "writes + prepare",
              "barrier B wait", "total"])
    if algo == native.MIOC_ALGO_FUSED:
        for q, nm in enumerate(names):
            print(f"{nm:28s} cycles/step median {np.median(st[:, q]):8.0f}  p10 {np.percentile(st[:, q], 10):8.0f}  p90 {np.percentile(st[:, q], 90):8.0f}")
    else:  # per wave: rows 8k + w
        nb = min(K, 512)
        st = np.array(buf, dtype=np.int64).reshape(4096, 8) / (cfg.nt - 1)
        for w in range(8):
            sw = st[[8 * b + w for b in range(nb)]]
            if not sw[:, 7].any():
                continue
            print(f"wave {w}: " + "  ".join(f"{nm.split()[0]} {np.median(sw[:, q]):6.0f}" for q, nm in enumerate(names)))
