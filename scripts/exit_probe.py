"""Control for the rocprofv3 exit SIGSEGV: a minimal GPU program (torch tensor on the device, optionally a libmioc
context created, used and destroyed) that writes /proc/self/maps at interpreter exit to $MIOC_EXIT_MAPS.
Usage: python scripts/exit_probe.py [torch|mioc|mioc_nocoop]
(mioc: C5 at K = 1 runs k_fsep2 in row segments, a cooperative launch; mioc_nocoop: the same DP as one ordinary
launch)"""
import atexit
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd"), ROOT]


def dump():
    path = os.environ.get("MIOC_EXIT_MAPS")
    if path:
        with open("/proc/self/maps") as f, open(path, "w") as g:
            g.write(f.read())


atexit.register(dump)
import torch  # noqa: E402

x = torch.ones(1024, device="cuda")
print("torch sum", float(x.sum()))
mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
if mode.startswith("mioc"):
    from mioc import native  # noqa: E402
    from mioc.synth import CONFIGS, make_inputs  # noqa: E402
    cfg = CONFIGS["C5"]
    lt, df, uo = make_inputs(cfg, nt=64)
    with native.Context(0) as ctx:
        ctx.set_levels(lt)
        ctx.set_cost(cfg.p, cfg.beta)
        if mode == "mioc_nocoop":  # one workgroup per subproblem: an ordinary launch, no cooperative one
            ctx.set_option(native.MIOC_OPT_FSEP_SEGMENTS, 1)
        ctx.bellman(df, uo, cfg.B, cfg.dt)
        ctx.synchronize()
        print("mioc algo", ctx.last_algo())
print("done", flush=True)
