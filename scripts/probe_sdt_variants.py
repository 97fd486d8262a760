"""Average k_sdt_step time per launch for library variants and batch sizes (C4 inputs, truncated nt).
Usage: python scripts/probe_sdt_variants.py NT LIB [LIB ...]   (each LIB run in its own process)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")


def one(nt, lib, Ks):
    os.environ["MIOC_LIB"] = lib
    sys.path.insert(0, PKG); sys.path.insert(0, ROOT)
    import numpy as np, torch
    from mioc import native
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS["C4"]
    lt = cfg.levels()
    out = {}
    for K in Ks:
        ins = [make_inputs(cfg, k=k, nt=nt, levels=lt) for k in range(K)]
        ddf = torch.tensor(np.ascontiguousarray(np.stack([d.T for _, d, _ in ins])), dtype=torch.float64, device="cuda")
        duo = torch.tensor(np.ascontiguousarray(np.stack([u.T for _, _, u in ins])), dtype=torch.float64, device="cuda")
        du = torch.empty_like(ddf); dphi = torch.empty(K, dtype=torch.float64, device="cuda")
        ctx = native.Context(0); ctx.set_levels(lt); ctx.set_cost(1, cfg.beta)
        ctx.set_option(native.MIOC_OPT_TIMING, 1)
        for rep in range(2):
            ctx.reset_stats()
            ctx.bellman_batch_tensors(ddf, duo, cfg.B, cfg.dt)
            ctx.backtrack_batch_tensors(cfg.B, du, dphi)
            ctx.synchronize()
        ms, n, name = ctx.kernel_stats(0)
        out[K] = {"kernel": name, "us_per_launch": round(1e3 * ms / n, 3), "us_per_subproblem_step": round(1e3 * ms / n / K, 3),
                  "phi": dphi.cpu().numpy().tolist()[:2], "diag": ctx.diagnostics()[:2]}
        ctx.close()
    print(json.dumps({"lib": os.path.basename(lib), "nt": nt, "res": out}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one(int(sys.argv[2]), sys.argv[3], [int(k) for k in sys.argv[4].split(",")])
    else:
        nt = int(sys.argv[1])
        for lib in sys.argv[2:]:
            r = subprocess.run([sys.executable, __file__, "--one", str(nt), lib, "1,2,4"], timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)
