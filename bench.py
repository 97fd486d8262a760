"""Benchmark: bellman_TRM! subproblems/sec on the BASELINE roofline config (C4) -- MI355X.

A "step" is one pass of the hot path over one batch of synthetic input: per rank, `--batch`
independent subproblems (default 1), each a full bellman_TRM! (DP over nt=65536 steps x 4096 levels
x B+1=257 budget rows) followed by eval_u_TRM! (backtrack), inputs already resident in HBM.

Alongside the headline it measures the batch config C5 (`batch`: `--batch-size` random restarts of the
36-level heat-shaped subproblem per GPU, the fused small-state DP), the same config at a fixed total
(`batch_strong`: `--batch-total` restarts split over the ranks, strong scaling) and the p=Inf variant of C4.

Multi-GPU: `python bench.py --gpus N` launches N ranks itself (one process per GPU, before anything
touches a GPU); under torchrun it uses the given RANK / WORLD_SIZE.  The problem descriptor is broadcast
once over RCCL, each rank solves its own block of every step's global batch (weak scaling: the per-GPU
work is fixed, no data-path collective), and the controls (uint16 level ranks from the library) plus Φ*
are gathered to rank 0 over RCCL at the end of every step.  `value` = subproblems of all ranks / the
max-over-ranks time.

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel, measured with HIP events on the
library's stream; `roofline_valu` gives the FP64-VALU view; `cpu_baseline` times the C restatement of the
reference loop (oracle/) on a bounded sample, on this job's host cores.

`--solver oracle --backend gloo` (CPU only, tests): the same launcher, sharding and gather, with the CPU
oracle as the per-rank solver on truncated inputs -- the product path on GPUs is libmioc.
"""
import argparse
import json
import math
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md
FP64_VALU_PEAK_TOPS = 39.3     # 256 CU x 64 FP64 lanes/clk x 2.4 GHz (78.6 TFLOP/s counts an FMA as 2)
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix, AMD spec (dense; the guide tabulates no FP64 MFMA row)
METRIC = "bellman_TRM! subproblems/sec (nt=65536, 4096 levels, budget=256) + HBM GB/s"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--p", default=None, help="override p: 1 or inf")
    ap.add_argument("--batch", type=int, default=1, help="subproblems per rank per step (headline config)")
    ap.add_argument("--total", type=int, default=0,
                    help="headline config: subproblems per step in total, split over the ranks (strong scaling; "
                         "default 0: --batch per rank, weak scaling)")
    ap.add_argument("--nt", type=int, default=None, help="truncate nt (profiling passes only; not a bench line)")
    ap.add_argument("--variant", default="pinf", help="extra p=Inf line on the same config ('' or none to skip)")
    ap.add_argument("--batch-config", default="C5", help="the batch line's config ('none' to skip)")
    ap.add_argument("--batch-size", type=int, default=1024, help="batch line: subproblems per rank per step")
    ap.add_argument("--batch-total", type=int, default=1024,
                    help="strong-scaling batch line (batch_strong): this many subproblems per step in total, split "
                         "over the ranks (0 to skip)")
    ap.add_argument("--shard8", type=int, default=1,
                    help="one GPU: also time the 1/8 shard of --batch-total (the per-rank work of the strong-scaling "
                         "batch at 8 GPUs), as the projection batch_shard8 (0 to skip)")
    ap.add_argument("--p2-batch-config", default="C5",
                    help="the batch line at p=2 (the reference's heat configuration, multi-trust.jl:193-195; "
                         "'none' to skip)")
    ap.add_argument("--pmc-valu", default=None,
                    help="a rocprofv3 --pmc CSV (SQ_INSTS_VALU, SQ_WAVES, ...) of THIS build over the same bench "
                         "command: adds counter-backed VALU figures to each line's roofline_valu")
    ap.add_argument("--pinf-batch-config", default="C2",
                    help="the p=Inf batch line's config (the reference's main() runs C1-C3 at p=Inf; 'none' to skip)")
    ap.add_argument("--single-configs", default="C2,C3",
                    help="one-subproblem lines (BASELINE configs 2 and 3, the reference's main() presets "
                         "multi-trust.jl:185-190) with their roofline and CPU baseline ('none' to skip)")
    ap.add_argument("--heat-restarts", type=int, default=4096,
                    help="PDE heat gradient line (SURVEY §8 f4): restarts per rank per step (0 to skip)")
    ap.add_argument("--heat-n", type=int, default=17, help="heat line: P1 grid side (N = n^2 dofs)")
    ap.add_argument("--heat-nt", type=int, default=500, help="heat line: time steps (example_heat.jl nt)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5, help="recursion steps timed for the C4 CPU baseline")
    ap.add_argument("--solver", default="native", choices=["native", "oracle"],
                    help="oracle: CPU test double for the launcher / sharding tests (no GPU)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------------
# launcher: one process per GPU, started before anything touches a GPU (no exec from a GPU process)
# ------------------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args):
    port = str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


# ------------------------------------------------------------------------------------------------------
# per-rank solvers
# ------------------------------------------------------------------------------------------------------
class NativeSolver:
    """libmioc (the product path): inputs resident in HBM, batched bellman + backtrack, ranks on device."""

    def __init__(self, device, levels, p, beta, torch):
        from mioc import native
        self.torch, self.native = torch, native
        self.device = device
        self.ctx = native.Context(device)
        self.ctx.set_levels(levels)
        self.ctx.set_cost(p, beta)
        self.ctx.set_option(native.MIOC_OPT_TIMING, 1)

    def load(self, dfs, uos, nsets, K, M):
        torch = self.torch
        nt = dfs[0].shape[1]
        # (sets, K, nt, nx) C-contiguous: each subproblem's nx x nt block column-major (mioc_bellman_batch_device)
        self.d_df = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in dfs])), dtype=torch.float64,
                                 device=self.device).reshape(nsets, K, nt, M).contiguous()
        self.d_uo = torch.tensor(np.ascontiguousarray(np.stack([d.T for d in uos])), dtype=torch.float64,
                                 device=self.device).reshape(nsets, K, nt, M).contiguous()
        self.d_u = torch.empty((K, nt, M), dtype=torch.float64, device=self.device)
        self.d_phi = torch.empty(K, dtype=torch.float64, device=self.device)
        self.d_st = torch.empty(K, dtype=torch.int32, device=self.device)
        self.d_rk = torch.empty((K, nt), dtype=torch.int32, device=self.device)

    def solve(self, s, B, dt):
        self.ctx.bellman_batch_tensors(self.d_df[s], self.d_uo[s], B, dt)
        self.ctx.backtrack_batch_tensors(B, self.d_u, self.d_phi, self.d_st)

    def results(self):
        """(level ranks int16 [K, nt], Φ* [K]) on the device, after solve()."""
        self.ctx.ranks_tensor(self.d_rk)
        self.ctx.synchronize()
        return self.d_rk.to(self.torch.int16), self.d_phi

    def sync(self):
        self.ctx.synchronize()
        self.torch.cuda.synchronize(self.device)

    def reset(self):
        self.ctx.reset_stats()

    def finish(self, res):
        st = self.d_st.cpu().numpy()
        if np.any(st != 0):
            raise RuntimeError(f"infeasible subproblem status {st}")
        dom_ms, dom_n, dom_name = self.ctx.kernel_stats(0)
        walk_ms, walk_n, _ = self.ctx.kernel_stats(1)
        res.update(algo=self.ctx.last_algo(), dom_ms=dom_ms, dom_n=dom_n, dom_name=dom_name, walk_ms=walk_ms,
                   diag=self.ctx.diagnostics(), phi=self.d_phi.cpu().numpy().tolist())
        self.ctx.close()


class OracleSolver:
    """CPU test double (tests of the launcher / sharding / gather over gloo): the C restatement."""

    def __init__(self, device, levels, p, beta, torch):
        from oracle.oracle import Levels, OracleC, P_INF, P_ONE
        self.torch = torch
        self.oc = OracleC()
        self.lv = Levels(levels.nu, [tuple(int(x) for x in t) for t in levels.tuples])
        self.kind = P_INF if p == math.inf else P_ONE
        self.beta = beta
        self.nuval = levels.nuval

    def load(self, dfs, uos, nsets, K, M):
        self.dfs, self.uos, self.K = dfs, uos, K

    def solve(self, s, B, dt):
        rk, ph = [], []
        for k in range(self.K):
            df, uo = self.dfs[s * self.K + k], self.uos[s * self.K + k]
            phi, U = self.oc.bellman(self.lv, df, uo, B, self.kind, self.beta, dt)
            u, ps = self.oc.backtrack(self.lv, uo, phi, U, B, B)
            rk.append([int(np.flatnonzero((self.nuval == u[:, i]).all(axis=1))[0]) for i in range(u.shape[1])])
            ph.append(ps)
        self._r = (self.torch.tensor(rk, dtype=self.torch.int16), self.torch.tensor(ph, dtype=self.torch.float64))

    def results(self):
        return self._r

    def sync(self):
        pass

    def reset(self):
        pass

    def finish(self, res):
        res.update(algo=0, dom_ms=0.0, dom_n=0, dom_name="oracle", walk_ms=0.0, diag=[0] * 8,
                   phi=self._r[1].numpy().tolist())


# ------------------------------------------------------------------------------------------------------
def run(args, cfg_name, K, p_over, nt_over, rank, world, device, dist, torch, steps, warmup, total=None):
    """One config: `steps` timed + `warmup` untimed steps, each a global batch of world*K subproblems (weak
    scaling), or of `total` subproblems split over the ranks (strong scaling)."""
    from mioc.batch import gather_results, shard
    from mioc.synth import CONFIGS, make_inputs

    cfg = CONFIGS[cfg_name]
    p = cfg.p if p_over is None else (math.inf if p_over == "inf" else float(p_over))
    nt = cfg.nt if nt_over is None else nt_over
    levels = cfg.levels()
    B = cfg.B
    # descriptor: broadcast once from rank 0 (RCCL) -- seeds, sizes, parameters
    dev = torch.device("cpu") if args.backend == "gloo" else torch.device("cuda", device)
    desc = torch.tensor([cfg.seed_df, cfg.seed_u, nt, B, cfg.dt, cfg.beta, p if p != math.inf else -1.0],
                        dtype=torch.float64, device=dev)
    if world > 1:
        dist.broadcast(desc, src=0)
    seed_df, seed_u, nt, B, dt, beta, pv = desc.tolist()
    nt, B = int(nt), int(B)
    p = math.inf if pv < 0 else pv

    solver = (NativeSolver if args.solver == "native" else OracleSolver)(device, levels, p, beta, torch)
    nsets = warmup + steps
    dfs, uos = [], []
    G = world * K if total is None else total  # each step's global batch
    lo, hi = shard(G, world, rank)  # this rank's contiguous block of it
    for s in range(nsets):
        for b in range(lo, hi):
            _, df, uo = make_inputs(cfg, k=s * G + b, nt=nt, levels=levels)
            dfs.append(df)
            uos.append(uo)
    solver.load(dfs, uos, nsets, hi - lo, levels.M)
    gathered = []

    def step(s):
        solver.solve(s, B, dt)
        if world > 1:  # controls as level ranks (uint16 payload) + Φ*, gathered to rank 0 over RCCL
            r, ph = solver.results()
            gathered.append(gather_results(dist, r, ph, G, world, rank))

    for s in range(warmup):
        step(s)
    solver.sync()
    solver.reset()
    if world > 1:
        dist.barrier()
    solver.sync()
    t0 = time.perf_counter()
    for s in range(warmup, nsets):
        step(s)
    solver.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    res = dict(config=cfg_name, elapsed=elapsed, K=hi - lo, G=G, nt=nt, B=B, p=p, levels=levels, uo=uos[-1],
               steps=steps, world=world)
    if world > 1 and rank == 0:
        R, PH = gathered[-1]
        res["gathered_checksum"] = float(PH.double().sum().item()) + float(R.double().sum().item())
    elif world == 1:
        r, ph = solver.results()
        res["gathered_checksum"] = float(ph.double().sum().item()) + float(r.double().sum().item())
    solver.finish(res)
    return res


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


def pmc_traffic(kernel, cfg=None, K=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/roundN_pmc_traffic.json,
    made by scripts/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), or None."""
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "round*_pmc_traffic.json"))
    found = []
    for f in files:
        try:
            with open(f) as fh:
                ks = json.load(fh)["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        # entries recorded from a single-config pass are qualified "kernel@CFG"; plain names come from the default
        # bench passes, where each kernel belongs to one line (C4 headline / its p=Inf variant / the C5 batch).
        # A batch size qualifier first ("k_fsep2@C5x128": the grid-size split of scripts/pmc_traffic.py --qualify);
        # an unqualified "@CFG" entry is a batch pass's, so a one-subproblem line (K = 1) never takes it.  `kernel` is
        # the launched variant (kernel_stats names it), so no prefix matching.
        e = ks.get(f"{kernel}@{cfg}x{K}") if K else None
        if not e and (not K or K > 1):
            e = ks.get(f"{kernel}@{cfg}")
        if not e and cfg in (None, "C4", "C5"):
            e = ks.get(kernel)
        if e and "hbm_bytes_per_launch" in e:
            found.append((int(re.search(r"round(\d+)_", os.path.basename(f)).group(1)), e["hbm_bytes_per_launch"], f))
    if not found:
        return None, None
    _, b, f = max(found)
    return b, os.path.relpath(f, ROOT)


def roofline_of(res):
    """Algorithmic bytes / flops of the dominant kernel per launch (SURVEY §8 d), over its HIP-event time."""
    lv, B, K, nt = res["levels"], res["B"], res["K"], res["nt"]
    L, M = lv.L, lv.M
    avg_s = (res["dom_ms"] / 1e3) / max(1, res["dom_n"])
    steps = 1  # DP recursion steps per launch
    name = res["dom_name"]
    ncand_step = candidates_per_step(lv, res["uo"], B)
    note = None
    if name == "k_generic_step":
        # front in + front out (fp64) + compact U (uint16/uint8) per step, per subproblem
        ub = 1 if L <= 256 else 2
        bytes_per_launch = K * (B + 1) * L * (8 + 8 + ub)
        ops = 2.0 * K * ncand_step  # one v_add_f64 + one v_min_f64 per candidate
    elif name in ("k_sdt_step", "k_sdt_run"):
        # the same algorithmic traffic as the reference DP step: front in + front out + compact U, per step;
        # k_sdt_run is one persistent launch over all nt - 1 steps
        steps = (nt - 1) if name != "k_sdt_step" else 1
        bytes_per_launch = steps * K * (B + 1) * L * (8 + 8 + 2)
        # per pass and 8-point line: 14 merges (7 forward, 7 backward), each add + min + sub + cmp (4 FP64 ops) and the
        # near-tie count's v_addc
        ops = 1.0 * steps * K * (B + 1) * L * M * (14 / 8) * 5
        note = "separable transform VALU ops (5 per merge, 4 of them FP64); brute-force-equivalent candidates/s = " \
               f"{steps * K * ncand_step / avg_s:.4g}"
    elif name in ("k_fused_run", "k_fsep_run", "k_fsep2"):
        # one launch = every step of K subproblems; the value fronts never leave the CU's LDS, so the HBM bytes
        # the DP must move are U (one byte per cell), df and u_old in, and Φ_0 out for the backtrack's argmin
        steps = nt - 1
        bytes_per_launch = K * (steps * (B + 1) * L + nt * M * 16 + L * (B + 1) * 8)
        if name == "k_fused_run":
            ops = 2.0 * K * steps * ncand_step  # v_add_f64 + v_min_f64 per candidate
            note = "min-plus candidates: 2 FP64 ops each"
        elif name == "k_fsep2":
            # two lanes per row: x0 pass N1 lines x 2(N0-1) merges, x1 pass per column 2 x 2(H-1) local merges
            # + 2H cross-half merges (H = N1/2); 6 32-bit VALU ops per merge (add_sat, min, sad, cmp, cndmask, or)
            n0, n1 = len(lv.nu[0]), len(lv.nu[1])
            h = n1 // 2
            merges = n1 * 2 * (n0 - 1) + n0 * (4 * (h - 1) + 2 * h)
            ops = 6.0 * K * steps * (B + 1) * merges
            seg = res.get("diag", [0] * 9)[8] if len(res.get("diag", [])) > 8 else 1
            if seg and seg > 1:  # the segment boundaries' outbox rows: written once, read once per step
                bytes_per_launch += K * (seg - 1) * steps * (n0 + n1 - 2) * L * 8 * 2
            note = (f"separable transform VALU lane-ops ({merges} fixed-point merges x 6 per row, {seg} row "
                    f"segment(s) per subproblem); brute-force-equivalent candidates/s = "
                    f"{K * steps * ncand_step / avg_s:.4g}")
        else:
            n0 = len(lv.nu[0])
            merges = 2 * (n0 - 1) * L // n0 + 2 * (L // n0 - 1) * L // (L // n0)  # both passes, both sweeps
            ops = 4.0 * K * steps * (B + 1) * merges
            note = (f"separable transform FP64 ops ({merges} merges x 4 per row); brute-force-equivalent "
                    f"candidates/s = {K * steps * ncand_step / avg_s:.4g}")
        sur = K * (steps * (B + 1) * L * (8 + 8 + 1) + nt * M * 24)
        note = (note + "; " if note else "") + (
            f"SURVEY §8 d's Q (fronts through HBM) would be {sur / avg_s / 1e9:.1f} GB/s = "
            f"{sur / avg_s / 1e9 / HBM_PEAK_GBS:.3f} of peak: the fused DP keeps the fronts in LDS instead")
    elif name == "k_pyr_step":
        bytes_per_launch = K * (B + 1) * L * (8 + 8 + 2)
        smax = int(sum(max(v) - min(v) for v in lv.nu))
        ops = 1.0 * K * (B + 1) * L * (smax + 1) * (2 * M + 2)  # upper bound: every level, 2M min + 2 add
        note = "pyramid ops upper bound (all levels)"
    else:
        # k_pinf_recur: one launch per subproblem batch; reads the class table, writes R rows
        bw = int(min(B, sum(max(v) - min(v) for v in lv.nu))) + 1
        bytes_per_launch = K * nt * (bw * 8 + (B + 1) * 8)
        ops = 2.0 * K * (nt - 1) * (B + 1) * bw
        steps = nt - 1  # one launch runs the whole recursion
    ach = bytes_per_launch / avg_s / 1e9
    traffic, tsrc = pmc_traffic(name, res["config"], K)
    roof = {"bound": "hbm", "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None if traffic is None else round(traffic),
            "traffic_source": tsrc, "kernel": name,
            "avg_launch_us": round(avg_s * 1e6, 3), "bytes_per_launch": bytes_per_launch,
            "us_per_dp_step": round(avg_s * 1e6 / steps, 3)}
    # FP64 and 32-bit VALU ops issue at the same rate on gfx950 (16 lanes per SIMD per clock)
    valu = {"bound": "valu", "achieved": round(ops / avg_s / 1e12, 6), "peak": FP64_VALU_PEAK_TOPS,
            "unit": "T VALU lane-ops/s" if name == "k_fsep2" else "TFP64op/s",
            "frac": round(ops / avg_s / 1e12 / FP64_VALU_PEAK_TOPS, 6)}
    if note:
        valu["note"] = note
    pmc = pmc_valu_of(name, avg_s, steps)
    if pmc:
        valu.update(pmc)
    return roof, valu


PMC_VALU_FILE = None  # --pmc-valu: a rocprofv3 --pmc CSV of this build over the same bench command


def pmc_valu_of(kernel, avg_s, steps):
    """Counter-backed VALU figures of `kernel` from the --pmc-valu CSV (a separate rocprofv3 --pmc pass of THIS build
    over the same bench command; no committed file of an older build is ever used): the dispatches of `kernel` whose
    duration is within 20 % of this line's HIP-event launch time, averaged.  VALU instructions per wave and DP step
    (SQ_INSTS_VALU / SQ_WAVES / steps) and the SIMDs' VALU-busy fraction: SQ_ACTIVE_INST_VALU counts quad-cycles
    summed over every wave, GRBM_GUI_ACTIVE cycles summed over the 8 XCDs (MI355X_MICROARCH.md, rocprofv3 PMC), so
    busy = ΣSQ_ACTIVE_INST_VALU·4 / (4 SIMDs · CUs · GRBM_GUI_ACTIVE/8) over the whole chip, and the same over the CUs
    the launch occupies (min(256, workgroups)); the wave-time split ACTIVE_INST_ANY / WAIT_ANY / WAIT_INST_ANY
    (disjoint, summing to SQ_WAVE_CYCLES) where the pass has them."""
    import csv
    path, how = PMC_VALU_FILE, "--pmc-valu (this build)"
    if not path:
        # else the newest committed pass (profiles/roundN_pmc_valu_bench.csv, by round number), labelled as such: its
        # dispatches count only where their duration matches this run's within 20 %
        import glob
        import re
        files = glob.glob(os.path.join(ROOT, "profiles", "round*_pmc_valu_bench.csv"))
        if not files:
            return None
        path = max(files, key=lambda f: int(re.search(r"round(\d+)_", os.path.basename(f)).group(1)))
        how = "committed PMC pass (not this run; its dispatches are matched to this line's kernel time within 20 %)"
    per = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if kernel not in r["Kernel_Name"]:
                continue
            dur = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
            if abs(dur - avg_s) > 0.2 * avg_s:
                continue
            d = per.setdefault(r["Dispatch_Id"], {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["_wgs"] = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
    if not per:
        return None
    avg = {}
    for d in per.values():
        for k, v in d.items():
            avg[k] = avg.get(k, 0.0) + v / len(per)
    out = {"pmc_source": os.path.relpath(path, ROOT), "pmc_pass": how, "pmc_dispatches": len(per)}
    if avg.get("SQ_INSTS_VALU") and avg.get("SQ_WAVES"):
        out["pmc_valu_instructions_per_wave_step"] = round(avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"] / steps, 1)
    if avg.get("SQ_ACTIVE_INST_VALU") and avg.get("GRBM_GUI_ACTIVE"):
        simd_cycles = 4 * avg["GRBM_GUI_ACTIVE"] / 8  # per CU: 4 SIMDs x the kernel's cycles
        out["pmc_valu_busy_frac"] = round(4 * avg["SQ_ACTIVE_INST_VALU"] / (256 * simd_cycles), 4)
        ncu = min(256, max(1, int(avg.get("_wgs", 256))))
        out["pmc_valu_busy_frac_active_cus"] = round(4 * avg["SQ_ACTIVE_INST_VALU"] / (ncu * simd_cycles), 4)
        out["pmc_active_cus"] = ncu
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc and avg.get("SQ_ACTIVE_INST_ANY") and avg.get("SQ_WAIT_ANY") and avg.get("SQ_WAIT_INST_ANY"):
        out["pmc_wave_time_split"] = {"issuing": round(avg["SQ_ACTIVE_INST_ANY"] / wc, 3),
                                      "waiting (waitcnt, barrier)": round(avg["SQ_WAIT_ANY"] / wc, 3),
                                      "issue-stalled": round(avg["SQ_WAIT_INST_ANY"] / wc, 3)}
    return out


def _cpu_info():
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    # this job's CPU share: OMP_NUM_THREADS where the launcher sets it (16 per GPU on the GPU box), else the
    # affinity mask
    threads = int(os.environ.get("OMP_NUM_THREADS") or aff)
    return model, aff, max(1, min(threads, aff))


def cpu_baseline(cfg_name, p_over, cpu_steps):
    """The reference recurrence (C restatement, oracle/) on the host: a bounded sample of the config."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle.oracle import OracleC, Levels, P_INF, P_ONE
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS[cfg_name]
    p = cfg.p if p_over is None else (math.inf if p_over == "inf" else float(p_over))
    kind = P_INF if p == math.inf else P_ONE
    model, aff, threads = _cpu_info()
    oc = OracleC()
    lut = None
    if p not in (1.0, math.inf):  # integer p: the reference loop with the host weight LUT (oracle_bellman)
        from mioc.native import cost_spec
        kind, p_int, lut = cost_spec(p, levels=cfg.levels())
    host = f"host: {model}, {aff} CPUs in the affinity mask, {threads} threads used (this job's CPU share)"
    if cfg.levels().L <= 64:
        # batch config: independent subproblems, one per thread (the reference is single-threaded per subproblem);
        # the sample is `threads` restarts at full nt, extrapolated to subproblems/s
        lt = cfg.levels()
        lv = Levels(lt.nu, [tuple(t) for t in lt.tuples])
        jobs = [make_inputs(cfg, k=10_000 + k, levels=lt)[1:] for k in range(threads)]

        def one(j):
            df, uo = j
            if lut is not None:
                return oc.bellman(lv, df, uo, cfg.B, kind, cfg.beta, cfg.dt, p_int=p_int, wtab=lut)[0][0, 0, 0]
            return oc.bellman_steps(lv, df, uo, cfg.B, kind, cfg.beta, cfg.dt, cfg.nt - 1)

        t0 = time.perf_counter()
        one(jobs[0])
        t1 = time.perf_counter() - t0
        # rounds of `threads` restarts until about 3 s of wall time (small restarts take milliseconds each)
        rounds = max(1, min(256, int(3.0 / max(t1, 1e-4))))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, jobs * rounds))
        tn = time.perf_counter() - t0
        return {"value": round(threads * rounds / tn, 6), "unit": "subproblems/s", "cores": threads, "kind": "port",
                "value_1thread": round(1.0 / t1, 6),
                "sample": f"{threads * rounds} full restarts (nt={cfg.nt}, L={lt.L}, B={cfg.B}, p="
                          f"{'inf' if p == math.inf else int(p)}) of the reference loop (C restatement), "
                          f"{threads} threads: {tn:.2f} s; one alone {t1:.3f} s; {host}"}
    per_step = {}
    for nthr, steps in ((1, cpu_steps), (threads, cpu_steps * max(1, min(threads, 8)))):
        lt, df, uo = make_inputs(cfg, nt=steps + 1)
        lv = Levels(lt.nu, [tuple(t) for t in lt.tuples])
        t0 = time.perf_counter()
        oc.bellman_steps(lv, df, uo, cfg.B, kind, cfg.beta, cfg.dt, steps, threads=nthr)
        per_step[nthr] = (time.perf_counter() - t0) / steps
    per_sub = {k: v * (cfg.nt - 1) for k, v in per_step.items()}
    return {"value": round(1.0 / per_sub[threads], 9), "unit": "subproblems/s", "cores": threads, "kind": "port",
            "value_1thread": round(1.0 / per_sub[1], 9),
            "sample": f"recursion steps of the reference loop (C restatement) at L={lt.L}, B={cfg.B}: "
                      f"{cpu_steps} steps on 1 thread ({per_step[1]:.3f} s/step) and "
                      f"{cpu_steps * max(1, min(threads, 8))} steps on {threads} OpenMP threads "
                      f"({per_step[threads]:.3f} s/step), extrapolated x{cfg.nt - 1}; {host}"}


def heat_line(args, rank, world, device, dist, torch):
    """The PDE heat objective's eval_f + eval_df (PDEObjective.jl:129-199) for K restarts per rank per step on the
    device (mioc_heat_eval_device, one k_heat_run launch), timed like the DP lines; HIP events on the library's
    stream give the kernel's own time for the MFMA roofline."""
    from mioc import native
    from mioc.heat import HeatProblem
    K, nt = args.heat_restarts, args.heat_nt
    steps = max(args.steps, 3)
    hp = HeatProblem(n=args.heat_n, nt=nt)
    ctx = native.Context(device)
    hp.setup(ctx)
    g = torch.Generator().manual_seed(1234 + rank)
    xs = [torch.randint(0, 6, (K, nt, 2), generator=g).double().to(f"cuda:{device}") for _ in range(2)]
    J = torch.empty(K, dtype=torch.float64, device=f"cuda:{device}")
    df = torch.empty_like(xs[0])
    st = torch.cuda.ExternalStream(ctx.stream(), device=f"cuda:{device}")
    for w in range(max(1, args.warmup)):
        ctx.heat_eval_tensors(xs[w % 2], J, df)
    ctx.synchronize()
    if world > 1:
        dist.barrier()
    ctx.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record(st)
    for s in range(steps):
        ctx.heat_eval_tensors(xs[s % 2], J, df)
    ev[1].record(st)
    ctx.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    kern_s = ev[0].elapsed_time(ev[1]) / 1e3 / steps
    N, Np = hp.N, (hp.N + 15) // 16 * 16
    flops = 3 * 2.0 * N * N * nt * K       # S^-1 z, M v (forward), S^-T r (adjoint): one N x N matvec each per step
    hbm = K * nt * (2 * Np * 8 + 2 * 2 * 8)  # Gy scratch written + read, x in + df out
    ach = flops / kern_s / 1e12
    traffic, tsrc = pmc_traffic("k_heat_run", "HEAT")
    line = {"config": {"workload": f"HEAT: example_heat.jl objective, N={N} dofs (P1 {args.heat_n}x{args.heat_n} "
                                   f"stand-in mesh), nx=2, nt={nt}, {K} restart(s) per GPU per step: eval_f + eval_df",
                       "parallelism": f"dp{world} (independent restarts)"},
            "value": round(world * K * steps / elapsed, 3), "unit": "gradient evaluations/s", "n_gpus": world,
            "scaling": "weak", "steps": steps, "ms_per_step": round(1e3 * elapsed / steps, 3),
            "algorithm": {"implicit-Euler state + adjoint on FP64 MFMA, LDS-resident columns": "k_heat_run"},
            "checksum": float(J.sum().item()) + float(df.sum().item()),
            "roofline": {"bound": "mfma", "achieved": round(ach, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 6),
                         "traffic": None if traffic is None else round(traffic), "traffic_source": tsrc,
                         "kernel": "k_heat_run", "avg_launch_us": round(kern_s * 1e6, 3),
                         "flops_per_launch": flops, "hbm_bytes_per_launch": hbm,
                         "hbm_frac": round(hbm / kern_s / 1e9 / HBM_PEAK_GBS, 6)}}
    ctx.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = heat_cpu_baseline(hp)
    return line


def heat_cpu_baseline(hp):
    """The reference's heat gradient (LU restatement, oracle/heat_oracle.py) on the host: restarts over a pool of
    single-threaded worker processes (spawned, BLAS at 1 thread each) for about 3 s."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor

    from oracle.heat_oracle import HeatOracle, eval_batch
    model, aff, threads = _cpu_info()
    mats = (hp.M_invA, hp.M_invF, hp.M, hp.state0, hp.yd)
    o = HeatOracle(*mats, hp.T0, hp.T1, hp.gamma)
    rng = np.random.default_rng(7)
    x0 = rng.integers(0, 6, size=(2, hp.nt)).astype(np.float64)
    t0 = time.perf_counter()
    o.eval(x0)
    t1 = time.perf_counter() - t0
    per = max(1, min(64, int(3.0 / max(t1, 1e-4))))  # restarts per worker: about 3 s each
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    for k in saved:
        os.environ[k] = "1"
    try:
        with ProcessPoolExecutor(threads, mp_context=mp.get_context("spawn")) as ex:
            list(ex.map(eval_batch, [(mats, hp.T0, hp.T1, hp.gamma, [x0])] * threads))  # start-up, untimed
            jobs = [(mats, hp.T0, hp.T1, hp.gamma, [x0] * per)] * threads
            t0 = time.perf_counter()
            list(ex.map(eval_batch, jobs))
            tn = time.perf_counter() - t0
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {"value": round(threads * per / tn, 3), "unit": "gradient evaluations/s", "cores": threads,
            "kind": "port", "value_1thread": round(1.0 / t1, 3),
            "sample": f"{threads * per} eval_f + eval_df of the heat objective (N={hp.N}, nt={hp.nt}; numpy/scipy "
                      f"LU restatement, one LAPACK triangular-solve pair per step) over {threads} single-threaded "
                      f"worker processes: {tn:.2f} s (matrix set-up per worker included); one alone {t1:.3f} s; "
                      f"host: {model}, {aff} CPUs in the affinity mask"}


def summary(out):
    """A compact view of every line (value, ms per step, roofline fraction, CPU baseline), the JSON line's last key."""
    def brief(d):
        r = {"value": d.get("value"), "unit": d.get("unit"), "ms_per_step": d.get("ms_per_step")}
        if isinstance(d.get("roofline"), dict):
            r["frac"] = d["roofline"].get("frac")
            r["bound"] = d["roofline"].get("bound")
            r["kernel"] = d["roofline"].get("kernel")
        if isinstance(d.get("cpu_baseline"), dict):
            r["cpu_value"] = d["cpu_baseline"].get("value")
        if "projected_8gpu_speedup" in d:
            r["projected_8gpu_speedup"] = d["projected_8gpu_speedup"]
        return r
    sm = {"C4": brief(out)}
    for key, name in (("variant_p_inf", "C4_p_inf"), ("batch", "batch"), ("batch_strong", "batch_strong"),
                      ("batch_shard8", "batch_shard8"), ("batch_p2", "batch_p2"), ("batch_p_inf", "batch_p_inf"),
                      ("batch_heat", "heat")):
        if key in out:
            sm[name] = brief(out[key])
    for key in out:
        if key.startswith("single_"):
            sm[key] = brief(out[key])
    return sm


def workload(res):
    lv = res["levels"]
    counts = "x".join(str(len(v)) for v in lv.nu)
    kind = "product" if lv.L == int(np.prod([len(v) for v in lv.nu])) else "SOS1-filtered"
    return (f"{res['config']}: nt={res['nt']}, {lv.L} levels ({counts} {kind}), B={res['B']}, "
            f"p={'inf' if res['p'] == math.inf else int(res['p'])}, {res['K']} subproblem(s) per GPU per step")


def native_name(algo):
    return {1: "generic min-plus sweep", 2: "p=Inf exact collapse", 3: "p=1 exact L1-ball pyramid",
            4: "p=1 separable L1 transform, certified argmin", 5: "fused small-state DP (front in LDS)",
            6: "fused separable DP (p=1, front in LDS, certified argmin)", 0: "oracle (CPU test double)"}.get(
        algo, str(algo))


def _exit_maps():
    """MIOC_EXIT_MAPS=path: write /proc/self/maps there at interpreter exit (before the C library's exit handlers
    run), so that the PCs of a crash inside exit() can be mapped to libraries (the rocprofv3 exit
    SIGSEGV)."""
    path = os.environ.get("MIOC_EXIT_MAPS")
    if not path:
        return
    import atexit

    def dump():
        try:
            with open("/proc/self/maps") as f, open(path, "w") as g:
                g.write(f.read())
        except OSError:
            pass
    atexit.register(dump)


def main():
    global PMC_VALU_FILE
    _exit_maps()
    args = parse()
    PMC_VALU_FILE = args.pmc_valu
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    device = local
    res = run(args, args.config, args.batch, args.p, args.nt, rank, world, device, dist, torch, args.steps,
              args.warmup, total=args.total or None)
    variant = batch = None
    if args.variant == "pinf" and args.p is None and args.nt is None and math.isfinite(res["p"]):
        r2 = run(args, args.config, args.batch, "inf", None, rank, world, device, dist, torch,
                 max(args.steps, 3), args.warmup)
        roof2, valu2 = roofline_of(r2)
        variant = {"p": "inf", "value": round(r2["G"] * r2["steps"] / r2["elapsed"], 6),
                   "unit": "subproblems/s", "ms_per_step": round(1e3 * r2["elapsed"] / r2["steps"], 3),
                   "algorithm": native_name(r2["algo"]), "roofline": roof2, "roofline_valu": valu2,
                   "backtrack_ms": round(r2["walk_ms"] / max(1, r2["steps"]), 3)}
        if args.solver == "native" and len(r2.get("diag", [])) > 9:  # mioc_diagnostics[9]
            variant["walk"] = "serial" if r2["diag"][9] < 0 else "segmented"
            variant["walk_serial_fallbacks"] = max(0, int(r2["diag"][9]))
        if rank == 0 and world == 1 and not args.no_cpu_baseline and args.solver == "native":
            variant["cpu_baseline"] = cpu_baseline(args.config, "inf", args.cpu_steps)
    def batch_line(cfg_name, total=None, p_over=None, min_steps=3):
        r3 = run(args, cfg_name, args.batch_size, p_over, None, rank, world, device, dist, torch,
                 max(args.steps, min_steps), args.warmup, total=total)
        line = {"config": {"workload": workload(r3), "parallelism": f"dp{world} (independent restarts)",
                           "global_batch": r3["G"], "per_rank": r3["K"]},
                "value": round(r3["G"] * r3["steps"] / r3["elapsed"], 3), "unit": "subproblems/s",
                "n_gpus": world, "scaling": "weak" if total is None else "strong", "steps": r3["steps"],
                "ms_per_step": round(1e3 * r3["elapsed"] / r3["steps"], 3),
                "algorithm": {native_name(r3["algo"]): r3["dom_name"]},
                "checksum": r3.get("gathered_checksum")}
        if args.solver == "native":
            if r3["algo"] == 2:
                line["backtrack_ms"] = round(r3["walk_ms"] / max(1, r3["steps"]), 3)
            else:
                line["exact_scan_targets"] = {"near_tie": r3["diag"][0], "out_of_binade_or_few": r3["diag"][1]}
            line["roofline"], line["roofline_valu"] = roofline_of(r3)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg_name, p_over, args.cpu_steps)
        return line

    batch_pinf = heat = None
    if args.heat_restarts > 0 and args.nt is None and args.solver == "native" and args.backend == "nccl":
        heat = heat_line(args, rank, world, device, dist, torch)
    if args.batch_config not in ("", "none") and args.nt is None:
        batch = batch_line(args.batch_config)
    strong = None
    if args.batch_total > 0 and args.batch_config not in ("", "none") and args.nt is None:
        if batch is not None and world == 1 and args.batch_total == args.batch_size:
            strong = dict(batch, scaling="strong")  # one rank: the same workload as the weak line
        else:  # fixed total work split over the ranks (C5 x 1024 on 8 GPUs: 128 restarts per GPU)
            strong = batch_line(args.batch_config, total=args.batch_total)
            strong.pop("cpu_baseline", None)
    shard8 = None
    if (args.shard8 and world == 1 and args.batch_total >= 8 and args.batch_config not in ("", "none") and
            args.nt is None):
        # the per-rank share of the strong-scaling batch on an 8-GPU node, timed on this one GPU: a projection of the
        # 8-GPU speed-up (the ranks share nothing but the start broadcast and the final gather)
        shard8 = batch_line(args.batch_config, total=args.batch_total // 8)
        shard8.pop("cpu_baseline", None)
        shard8["projection"] = (f"one GPU running the 1/8 shard ({args.batch_total // 8} restarts) of the "
                                f"{args.batch_total}-restart strong-scaling batch; the 8-GPU speed-up it projects is "
                                f"the full batch's ms_per_step over this line's")
        full = strong if strong is not None else batch
        if full is not None and full["config"]["global_batch"] == args.batch_total:
            shard8["projected_8gpu_speedup"] = round(full["ms_per_step"] / shard8["ms_per_step"], 3)
    batch_p2 = None
    if args.p2_batch_config not in ("", "none") and args.nt is None:
        batch_p2 = batch_line(args.p2_batch_config, p_over="2")
        batch_p2["note"] = ("p = 2 weights (Σ|Δ|²)^(1/2) from a host LUT (Python pow; Julia's own ^ through "
                            "integration/MIOC.jl): the reference's heat configuration (multi-trust.jl:193-195)")
    if args.pinf_batch_config not in ("", "none") and args.nt is None:
        batch_pinf = batch_line(args.pinf_batch_config)
    singles = {}
    if args.single_configs not in ("", "none") and args.nt is None:
        # one subproblem per GPU per step of the reference's own main() presets (doubletank, vanderpol at p = Inf); a
        # stream of 20 subproblems (0.5-1.7 ms each), so that the end of the timed region -- the last backtrack, which
        # nothing overlaps, and the synchronisation -- weighs as in a stream rather than a third of the total (3 steps)
        for cname in args.single_configs.split(","):
            saved = args.batch_size
            args.batch_size = 1
            try:
                singles[cname] = batch_line(cname, min_steps=20)
            finally:
                args.batch_size = saved
    if rank == 0:
        value = res["G"] * args.steps / res["elapsed"]
        out = {
            "metric": METRIC,
            "value": round(value, 6),
            "unit": "subproblems/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * res["elapsed"] / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.total else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded N(0,1) df, rand_func_int-shaped u_old; SURVEY §8 d)",
            "config": {"workload": workload(res),
                       "parallelism": f"dp{world} (independent subproblems" +
                                      ("; one GPU, no collective)" if world == 1 else
                                       "; RCCL broadcast of the problem, gather of the controls)")},
            "algorithm": {native_name(res["algo"]): res["dom_name"]},
            "checksum": res.get("gathered_checksum"),
        }
        if args.solver == "native":
            out["roofline"], out["roofline_valu"] = roofline_of(res)
            out["backtrack_ms"] = round(res["walk_ms"] / max(1, args.steps), 3)
            out["exact_scan_targets"] = {"near_tie": res["diag"][0], "direct_rows": res["diag"][1],
                                         "of_cells": res["K"] * (res["nt"] - 1) * (res["B"] + 1) * res["levels"].L,
                                         "note": "last bellman call (mioc_diagnostics[0..1])"}
        if variant:
            out["variant_p_inf"] = variant
        if batch:
            out["batch"] = batch
        if strong:
            out["batch_strong"] = strong
        if shard8:
            out["batch_shard8"] = shard8
        if batch_p2:
            out["batch_p2"] = batch_p2
        if batch_pinf:
            out["batch_p_inf"] = batch_pinf
        if heat:
            out["batch_heat"] = heat
        for cname, line in singles.items():
            out[f"single_{cname}"] = line
        if not args.no_cpu_baseline and world == 1 and args.nt is None and args.solver == "native":
            out["cpu_baseline"] = cpu_baseline(args.config, args.p, args.cpu_steps)
        out["summary"] = summary(out)  # last key: every sub-line in the tail of the output
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
