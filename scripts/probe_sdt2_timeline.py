"""Timeline of k_sdt_pair (the two-workgroups-per-row persistent separable DP, mioc_sdt2.hip) from the diagnostic
build libmioc_stamps_tl.so (`make stamps_tl`): per workgroup and for 32 of its items from the middle of the run,
s_memrealtime (100 MHz) at 8 points of an item: 0 start, 1 statistics written (before the drain and barrier 1 that
publish the previous item), 2 before the transform, 3 after the transform, 4 winners done (go() entered), 5 go()'s
polls matched and the next loads issued, 6 (= 5), 7 stores issued.  Prints the phase medians, the item period per workgroup and the skew between rows.
Usage: python scripts/probe_sdt2_timeline.py [nt]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
os.environ.setdefault("MIOC_LIB", os.path.join(PKG, "lib", "libmioc_stamps_tl.so"))
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)
from mioc import native  # noqa: E402
from mioc.synth import CONFIGS, make_inputs  # noqa: E402


def main():
    nt = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    _, df, uo = make_inputs(cfg, nt=nt, levels=lt)
    with native.Context(0) as ctx:
        ctx.set_levels(lt)
        ctx.set_cost(1, cfg.beta)
        ctx.set_option(native.MIOC_OPT_TIMING, 1)
        ctx.set_option(native.MIOC_OPT_SDT_PAIR, int(os.environ.get("SDT_PAIR", "1")))  # 1: 256 threads, 2: 512
        if int(os.environ.get("SDT_NB", "0")):  # staging buffers (MIOC_OPT_SDT_BUFFERS)
            ctx.set_option(native.MIOC_OPT_SDT_BUFFERS, int(os.environ["SDT_NB"]))
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        ctx.synchronize()
        ms, _, name = ctx.kernel_stats(0)
        print(f"{name}: {ms:.3f} ms for {nt - 1} steps = {1e3 * ms / (nt - 1):.3f} us/step; diag {ctx.diagnostics()}")
    lib = native.load_library()
    NB = 2 * cfg.B  # (workgroups)
    buf = np.zeros((1024, 32, 8), dtype=np.uint64)
    f = lib.mioc_debug_sdt2_timeline
    f.restype = ctypes.c_int32
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert f(buf.ctypes.data, 1024) == 0
    raw_unmet = (buf[:NB, :, 5] >> np.uint64(62)) & np.uint64(1)
    war_unmet = (buf[:NB, :, 5] >> np.uint64(61)) & np.uint64(1)
    buf[:NB, :, 5] &= np.uint64((1 << 61) - 1)
    print(f"go() first test unmet: RAW {raw_unmet.mean():.3f}, WAR {war_unmet.mean():.3f} of the items")
    t = buf[:NB].astype(np.float64) * 0.01  # us (100 MHz)
    bx = np.zeros((1024, 32, 4), dtype=np.uint64)
    fx = lib.mioc_debug_sdt2_timeline_x
    fx.restype = ctypes.c_int32
    fx.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fx(bx.ctypes.data, 1024) == 0
    out = os.environ.get("TL_SAVE")  # the raw stamps for offline analysis (blocks x items x points, us)
    if out:
        np.save(out, t)
        np.save(out.replace(".npy", "_x.npy"), bx[:NB])
    d = np.diff(t, axis=2)
    names = ["start -> stats written", "drain + barrier 1 + head value", "transform", "winners", "poll wait + issue",
             "-", "orders + scans + gather + stores"]
    for q, nm in enumerate(names):
        x = d[:, :, q].ravel()
        print(f"{nm:34s} median {np.median(x):7.3f}  p10 {np.percentile(x, 10):7.3f}  p90 {np.percentile(x, 90):7.3f} us")
    per = np.diff(t[:, :, 0], axis=1).ravel()  # item period of one workgroup (two DP steps)
    print(f"item period per workgroup: median {np.median(per):.3f} us (two DP steps: {np.median(per) / 2:.3f} us/step)")
    item = np.median(t[:, :, 7] - t[:, :, 0])
    print(f"item latency start -> stores issued: median {item:.3f} us")
    # rows: block b -> row by the kernel's XCD-aware map (NR % 8 == 0)
    R = cfg.B
    rid0 = np.arange(R)
    row = (rid0 & 7) * (R >> 3) + (rid0 >> 3) + 1
    st0 = t[:R, 0, 0]  # parity-0 workgroups, first stamped item
    order = np.argsort(row)
    sk = np.diff(st0[order])
    print(f"skew row c vs c-1 (parity 0, same item): median {np.median(sk):.3f} us, total {np.sum(sk):.1f} us")
    # per row (parity 0): the phases of rows 1, 2, 3, B/2 and B
    blk = {int(r): int(b) for b, r in enumerate(row)}
    for r in (1, 2, 3, R // 2, R):
        b = blk[r]
        ph = " ".join(f"{np.median(d[b, :, q]):6.2f}" for q in range(7))
        print(f"row {r:4d}: phases {ph}  period {np.median(np.diff(t[b, :, 0])):6.2f} us  "
              f"unmet RAW {raw_unmet[b].mean():.2f} WAR {war_unmet[b].mean():.2f}")


if __name__ == "__main__":
    main()
