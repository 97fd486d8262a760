"""C4 at p = Inf (one subproblem, full L and B, nt from argv) across library builds, each in its own process:
k_pinf_recur time per launch (HIP events), k_pinf_prep's, the whole bellman + backtrack wall time, and a digest of u / Φ* at three
budgets, which must agree across builds.  Usage: python scripts/probe_pinf_c4.py NT LIB [LIB ...]
(PINF_CFG=C1 / C2 / C3: that config instead of C4; NT 0: the config's own nt)"""
import hashlib, json, math, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")


def one(nt, lib):
    os.environ["MIOC_LIB"] = lib
    sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
    import numpy as np
    from mioc import native
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS[os.environ.get("PINF_CFG", "C4")]
    nt = nt or cfg.nt
    lt = cfg.levels()
    _, df, uo = make_inputs(cfg, nt=nt, levels=lt)
    with native.Context(0) as ctx:
        ctx.set_levels(lt); ctx.set_cost(math.inf, cfg.beta)
        ctx.set_option(native.MIOC_OPT_TIMING, 1)
        best, wall, prep = None, None, None
        for _ in range(3):
            ctx.reset_stats()
            t0 = time.perf_counter()
            ctx.bellman(df, uo, cfg.B, cfg.dt)
            ctx.synchronize()
            w = time.perf_counter() - t0
            ms, n, name = ctx.kernel_stats(0)
            pms, pn, _ = ctx.kernel_stats(2)  # k_pinf_prep
            best = ms / n if best is None else min(best, ms / n)
            prep = pms / max(pn, 1) if best == ms / n else prep
            wall = w if wall is None else min(wall, w)
        h = hashlib.sha256()
        try:  # (a timing-only build with wrong tables may have no finite path: digest "error")
            for Bp in (cfg.B, cfg.B // 2, 7):
                u, phi, _ = ctx.backtrack(Bp)
                h.update(np.ascontiguousarray(u).tobytes()); h.update(np.float64(phi).tobytes())
        except native.MiocNativeError:
            h = None
        print(json.dumps({"lib": os.path.basename(lib), "nt": nt, "kernel": name, "ms": round(best, 3),
                          "us_per_step": round(1e3 * best / (nt - 1), 4), "prep_ms": round(prep, 3),
                          "bellman_wall_ms": round(1e3 * wall, 3),
                          "digest": h.hexdigest()[:16] if h else "error"}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one(int(sys.argv[2]), sys.argv[3])
    else:
        for lib in sys.argv[2:]:
            r = subprocess.run([sys.executable, __file__, "--one", sys.argv[1], lib], timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)
