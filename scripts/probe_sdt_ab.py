"""A/B timing of k_sdt_run (C4 inputs at full L and B, truncated nt) across library builds, each in its own process.
Prints per library: µs per DP step (HIP events, best of REPS calls) and a digest of u / Φ* at three budgets and of
the argmin tables of a few steps, which must agree across builds.
Usage: python scripts/probe_sdt_ab.py NT LIB [LIB ...]   (SDT_NB=n: staging buffers; a LIB may be repeated to
interleave runs of the same build, LIB#tag only labels the run)"""
import hashlib, json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
REPS = 3


NB = int(os.environ.get("SDT_NB", "0"))  # staging buffers (MIOC_OPT_SDT_BUFFERS), 0: the library default


def one(nt, spec):
    lib = spec.partition("#")[0]
    os.environ["MIOC_LIB"] = lib
    sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
    import numpy as np
    from mioc import native
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    _, df, uo = make_inputs(cfg, nt=nt, levels=lt)
    with native.Context(0) as ctx:
        ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
        ctx.set_option(native.MIOC_OPT_TIMING, 1); ctx.set_option(native.MIOC_OPT_PERSIST, 1)
        if NB:
            ctx.set_option(native.MIOC_OPT_SDT_BUFFERS, NB)
        best = None
        for _ in range(REPS):
            ctx.reset_stats()
            ctx.bellman(df, uo, cfg.B, cfg.dt)
            ctx.synchronize()
            ms, n, name = ctx.kernel_stats(0)
            best = ms if best is None else min(best, ms)
        h = hashlib.sha256()
        for Bp in (cfg.B, cfg.B // 2, 7):
            try:  # (timing-only builds make wrong tables: their digest is "error")
                u, phi, _ = ctx.backtrack(Bp)
            except native.MiocNativeError:
                h.update(b"error")
                continue
            h.update(np.ascontiguousarray(u).tobytes()); h.update(np.float64(phi).tobytes())
        for i in (0, 1, nt // 2, nt - 3):
            h.update(np.ascontiguousarray(ctx.argmin_table(i), dtype=np.int32).tobytes())
        print(json.dumps({"lib": os.path.basename(spec), "nt": nt, "kernel": name, "ms": round(best, 3),
                          "us_per_step": round(1e3 * best / (nt - 1), 3), "diag": list(ctx.diagnostics()[:7]),
                          "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one(int(sys.argv[2]), sys.argv[3])
    else:
        nt = int(sys.argv[1])
        for lib in sys.argv[2:]:
            r = subprocess.run([sys.executable, __file__, "--one", str(nt), lib], timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)
