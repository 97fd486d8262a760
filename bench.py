"""Benchmark: bellman_TRM! subproblems/sec on the BASELINE roofline config (C4) -- MI355X.

A "step" is one pass of the hot path over one batch of synthetic input: per rank, `--batch`
independent subproblems (default 1), each a full bellman_TRM! (DP over nt=65536 steps x 4096 levels
x B+1=257 budget rows) followed by eval_u_TRM! (backtrack), inputs already resident in HBM.
Multi-GPU (torchrun, one process per GPU): the problem descriptor is broadcast once over RCCL, each
rank solves its own restarts (weak scaling, no data-path collective) and the controls (as uint16
level ranks) plus Φ* are gathered to rank 0 over RCCL at the end of every step.

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel, measured with HIP events on
the library's stream; `roofline_valu` gives the FP64-VALU view (the p=1 sweep is VALU-bound);
`cpu_baseline` times the C restatement of the reference loop (oracle/) on a bounded sample.
"""
import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md
FP64_VALU_PEAK_TOPS = 39.3     # 256 CU x 64 FP64 lanes/clk x 2.4 GHz (78.6 TFLOP/s counts an FMA as 2)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--p", default=None, help="override p: 1 or inf")
    ap.add_argument("--batch", type=int, default=1, help="subproblems per rank per step")
    ap.add_argument("--nt", type=int, default=None, help="truncate nt (profiling passes only; not a bench line)")
    ap.add_argument("--variant", default="pinf", help="extra p=Inf line on the same config ('' to skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5, help="recursion steps timed for the CPU baseline")
    return ap.parse_args()


def candidates_per_step(levels, uo, B):
    """Exact N_cand = sum_l L * max(0, B+1-b̃(l,i)) per step (SURVEY §8 d), averaged over steps."""
    nv = levels.nuval
    tot = 0
    nt = uo.shape[1]
    for s in range(0, nt - 1, 512):
        e = min(nt - 1, s + 512)
        bt = np.abs(nv[:, :, None] - uo[None, :, s:e]).sum(axis=1)  # L x steps
        tot += np.maximum(0, B + 1 - bt).sum()
    return levels.L * tot / max(1, nt - 1)


def run(args, rank, world, device, dist, torch):
    from mioc import native
    from mioc.batch import gather_results, level_ranks, shard
    from mioc.synth import CONFIGS, make_inputs

    cfg = CONFIGS[args.config]
    p = cfg.p if args.p is None else (math.inf if args.p == "inf" else float(args.p))
    nt = cfg.nt if args.nt is None else args.nt
    levels = cfg.levels()
    B = cfg.B

    # descriptor: broadcast once from rank 0 (RCCL) -- seeds, sizes, parameters
    desc = torch.tensor([cfg.seed_df, cfg.seed_u, nt, B, cfg.dt, cfg.beta, p if p != math.inf else -1.0],
                        dtype=torch.float64, device=device)
    if world > 1:
        dist.broadcast(desc, src=0)
    seed_df, seed_u, nt, B, dt, beta, pv = desc.tolist()
    nt, B = int(nt), int(B)
    p = math.inf if pv < 0 else pv

    ctx = native.Context(device)
    ctx.set_levels(levels)
    ctx.set_cost(p, beta)
    ctx.set_option(native.MIOC_OPT_TIMING, 1)

    K = args.batch
    nsets = args.warmup + args.steps
    dfs, uos = [], []
    lo, hi = shard(world * K, world, rank)  # this rank's contiguous block of each step's global batch
    for s in range(nsets):
        for b in range(lo, hi):
            k = s * world * K + b
            _, df, uo = make_inputs(cfg, k=k, nt=nt, levels=levels)
            dfs.append(df)
            uos.append(uo)
    # (sets, K, nt, nx) C-contiguous: each subproblem's nx x nt block column-major (mioc_bellman_batch_device)
    d_df = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64,
                        device=device).reshape(nsets, K, nt, -1).contiguous()
    d_uo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64,
                        device=device).reshape(nsets, K, nt, -1).contiguous()
    d_u = torch.empty((K, nt, levels.M), dtype=torch.float64, device=device)
    d_phi = torch.empty(K, dtype=torch.float64, device=device)
    d_st = torch.empty(K, dtype=torch.int32, device=device)
    nuval = torch.tensor(levels.nuval, dtype=torch.float64, device=device)

    def step(s):
        ctx.bellman_batch_tensors(d_df[s], d_uo[s], B, dt)
        ctx.backtrack_batch_tensors(B, d_u, d_phi, d_st)
        if world > 1:
            ctx.synchronize()
            # controls as level ranks (uint16 payload) + Φ*, gathered to rank 0 over RCCL
            gather_results(dist, level_ranks(d_u, nuval), d_phi, world * K, world, rank)

    for s in range(args.warmup):
        step(s)
    ctx.synchronize()
    torch.cuda.synchronize(device)
    ctx.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s in range(args.warmup, nsets):
        step(s)
    ctx.synchronize()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    st = d_st.cpu().numpy()
    if np.any(st != 0):
        raise RuntimeError(f"rank {rank}: infeasible subproblem status {st}")

    dom_ms, dom_n, dom_name = ctx.kernel_stats(0)
    walk_ms, walk_n, walk_name = ctx.kernel_stats(1)
    algo = ctx.last_algo()
    res = dict(elapsed=elapsed, K=K, nt=nt, B=B, p=p, algo=algo, dom_ms=dom_ms, dom_n=dom_n, dom_name=dom_name,
               walk_ms=walk_ms, walk_n=walk_n, walk_name=walk_name, levels=levels, uo=uos[-1],
               phi=d_phi.cpu().numpy().tolist(), diag=ctx.diagnostics())
    ctx.close()
    return res


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/roundN_pmc_traffic.json,
    made by scripts/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), or None."""
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "round*_pmc_traffic.json"))
    if not files:
        return None, None
    f = max(files, key=lambda x: int(re.search(r"round(\d+)_", os.path.basename(x)).group(1)))
    try:
        with open(f) as fh:
            e = json.load(fh)["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None, None
    if not e or "hbm_bytes_per_launch" not in e:
        return None, None
    return e["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)


def roofline_of(res, args):
    """Algorithmic bytes / flops of the dominant kernel per launch (SURVEY §8 d), over its HIP-event time."""
    lv, B, K, nt = res["levels"], res["B"], res["K"], res["nt"]
    L = lv.L
    avg_s = (res["dom_ms"] / 1e3) / max(1, res["dom_n"])
    steps = 1  # DP recursion steps per launch
    if res["dom_name"] == "k_generic_step":
        # front in + front out (fp64) + compact U (uint16/uint8) per step, per subproblem
        ub = 1 if L <= 256 else 2
        bytes_per_launch = K * (B + 1) * L * (8 + 8 + ub)
        ncand = K * candidates_per_step(lv, res["uo"], B)
        ops = 2.0 * ncand  # one v_add_f64 + one v_min_f64 per candidate
        roof_valu = {"bound": "valu", "achieved": ops / avg_s / 1e12, "peak": FP64_VALU_PEAK_TOPS,
                     "unit": "TFP64op/s", "frac": ops / avg_s / 1e12 / FP64_VALU_PEAK_TOPS,
                     "candidates_per_launch": ncand}
    elif res["dom_name"] in ("k_sdt_step", "k_sdt_run"):
        # the same algorithmic traffic as the reference DP step: front in + front out + compact U, per step;
        # k_sdt_run is one persistent launch over all nt - 1 steps
        steps = (nt - 1) if res["dom_name"] == "k_sdt_run" else 1
        bytes_per_launch = steps * K * (B + 1) * L * (8 + 8 + 2)
        M = lv.M
        # per pass and 8-point line: 20 merges (7 forward, 6 backward, 7 combine), each add + min + sub + cmp
        ops = 1.0 * steps * K * (B + 1) * L * M * (20 / 8) * 4
        ncand = steps * K * candidates_per_step(lv, res["uo"], B)
        roof_valu = {"bound": "valu", "achieved": ops / avg_s / 1e12, "peak": FP64_VALU_PEAK_TOPS,
                     "unit": "TFP64op/s", "frac": ops / avg_s / 1e12 / FP64_VALU_PEAK_TOPS,
                     "note": "separable transform FP64 ops (4 per merge); brute-force-equivalent candidates/s "
                             f"= {ncand / avg_s:.4g}"}
    elif res["dom_name"] == "k_pyr_step":
        # the same algorithmic traffic as the reference DP step: front in + front out + compact U
        bytes_per_launch = K * (B + 1) * L * (8 + 8 + 2)
        M = lv.M
        smax = int(sum(max(v) - min(v) for v in lv.nu))
        ops = 1.0 * K * (B + 1) * L * (smax + 1) * (2 * M + 2)  # upper bound: every level, 2M min + 2 add
        ncand = K * candidates_per_step(lv, res["uo"], B)
        roof_valu = {"bound": "valu", "achieved": ops / avg_s / 1e12, "peak": FP64_VALU_PEAK_TOPS,
                     "unit": "TFP64op/s", "frac": ops / avg_s / 1e12 / FP64_VALU_PEAK_TOPS,
                     "note": "pyramid ops upper bound (all levels); brute-force-equivalent candidates/s "
                             f"= {ncand / avg_s:.4g}"}
    else:
        # k_pinf_recur: one launch per subproblem batch; reads the class table, writes R rows
        bw = int(min(B, sum(max(v) - min(v) for v in lv.nu))) + 1
        bytes_per_launch = K * nt * (bw * 8 + (B + 1) * 8)
        ops = 2.0 * K * (nt - 1) * (B + 1) * bw
        roof_valu = {"bound": "valu", "achieved": ops / avg_s / 1e12, "peak": FP64_VALU_PEAK_TOPS,
                     "unit": "TFP64op/s", "frac": ops / avg_s / 1e12 / FP64_VALU_PEAK_TOPS}
    ach = bytes_per_launch / avg_s / 1e9
    traffic, tsrc = pmc_traffic(res["dom_name"])
    roof = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None if traffic is None else round(traffic),
            "traffic_source": tsrc, "kernel": res["dom_name"],
            "avg_launch_us": round(avg_s * 1e6, 3), "bytes_per_launch": bytes_per_launch,
            "us_per_dp_step": round(avg_s * 1e6 / steps, 3)}
    roof_valu = {k: (round(v, 6) if isinstance(v, float) else v) for k, v in roof_valu.items()}
    return roof, roof_valu


def cpu_baseline(args):
    """The reference recurrence (C restatement, oracle/) on the host: a bounded truncated sample."""
    from oracle.oracle import OracleC, Levels, P_INF, P_ONE
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS[args.config]
    p = cfg.p if args.p is None else (math.inf if args.p == "inf" else float(args.p))
    # single-thread (the reference is single-threaded Julia) and OpenMP over the target levels
    # on the host cores this job may use (OMP_NUM_THREADS on the GPU box; os.cpu_count() there is the machine's)
    threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
    kind = P_INF if p == math.inf else P_ONE
    oc = OracleC()
    per_step = {}
    for nthr, steps in ((1, args.cpu_steps), (threads, args.cpu_steps * max(1, min(threads, 8)))):
        lt, df, uo = make_inputs(cfg, nt=steps + 1)
        lv = Levels(lt.nu, [tuple(t) for t in lt.tuples])
        t0 = time.perf_counter()
        oc.bellman_steps(lv, df, uo, cfg.B, kind, cfg.beta, cfg.dt, steps, threads=nthr)
        per_step[nthr] = (time.perf_counter() - t0) / steps
    per_sub = {k: v * (cfg.nt - 1) for k, v in per_step.items()}
    return {"value": 1.0 / per_sub[threads], "unit": "subproblems/s", "cores": threads, "kind": "port",
            "value_1thread": 1.0 / per_sub[1],
            "sample": f"recursion steps of the reference loop (C restatement) at L={lt.L}, B={cfg.B}: "
                      f"{args.cpu_steps} steps on 1 thread ({per_step[1]:.3f} s/step) and "
                      f"{args.cpu_steps * max(1, min(threads, 8))} steps on {threads} OpenMP threads "
                      f"({per_step[threads]:.3f} s/step), extrapolated x{cfg.nt - 1}; host {platform.processor() or platform.machine()}, "
                      f"{os.cpu_count()} CPUs visible"}


def main():
    args = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = local
    res = run(args, rank, world, device, dist, torch)
    variant = None
    if args.variant == "pinf" and args.p is None and args.nt is None and math.isfinite(res["p"]):
        a2 = argparse.Namespace(**vars(args))
        a2.p = "inf"
        a2.steps = max(args.steps, 3)
        r2 = run(a2, rank, world, device, dist, torch)
        roof2, valu2 = roofline_of(r2, a2)
        variant = {"p": "inf", "value": round(world * r2["K"] * a2.steps / r2["elapsed"], 6),
                   "unit": "subproblems/s", "ms_per_step": round(1e3 * r2["elapsed"] / a2.steps, 3),
                   "algorithm": "p=Inf exact collapse (k_pinf_prep/recur/walk)", "roofline": roof2,
                   "roofline_valu": valu2, "backtrack_ms": round(r2["walk_ms"] / max(1, a2.steps), 3)}
    if rank == 0:
        roof, valu = roofline_of(res, args)
        value = world * res["K"] * args.steps / res["elapsed"]
        out = {
            "metric": "bellman_TRM! subproblems/sec (nt=65536, 4096 levels, budget=256) + HBM GB/s",
            "value": round(value, 6),
            "unit": "subproblems/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * res["elapsed"] / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded N(0,1) df, rand_func_int-shaped u_old; SURVEY §8 d)",
            "config": {"workload": f"{args.config}: nt={res['nt']}, 4096 levels (8^4 product), B={res['B']}, "
                                   f"beta=1e-3, p={'inf' if res['p'] == math.inf else int(res['p'])}, "
                                   f"{res['K']} subproblem(s) per GPU per step",
                       "parallelism": f"replicas x{world} (independent subproblems, RCCL gather of results)"},
            "algorithm": {native_name(res["algo"]): res["dom_name"]},
            "roofline": roof,
            "roofline_valu": valu,
            "backtrack_ms": round(res["walk_ms"] / max(1, args.steps), 3),
            "exact_scan_targets": {"near_tie": res["diag"][0], "direct_rows": res["diag"][1],
                                   "of_cells": res["K"] * (res["nt"] - 1) * (res["B"] + 1) * res["levels"].L,
                                   "note": "last bellman call (mioc_diagnostics[0..1])"},
        }
        if variant:
            out["variant_p_inf"] = variant
        if not args.no_cpu_baseline and world == 1 and args.nt is None:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def native_name(algo):
    return {1: "generic min-plus sweep", 2: "p=Inf exact collapse", 3: "p=1 exact L1-ball pyramid",
            4: "p=1 separable L1 transform, certified argmin"}.get(algo, str(algo))


if __name__ == "__main__":
    main()
