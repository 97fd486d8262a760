"""Sharding a batch of independent subproblems (random restarts / a Δ-sweep) over ranks.

SURVEY.md §8 (e): the path partitions at subproblem granularity, so there is no data-path collective.
Each rank solves one contiguous block of the batch on its own GPU. Rank 0 receives the controls, as
uint16 level ranks (the reference's `U` tuple, HelpFunctions.jl:74), and Φ* through `gather`. On GPUs
the backend is `nccl` (RCCL over xGMI); the CPU tests use `gloo`. The solver itself is the caller's:
`bench.py` passes the libmioc context.
"""
from __future__ import annotations


def shard(n_total, world, rank):
    """[lo, hi) of the contiguous block of `n_total` subproblems owned by `rank`; sizes differ by <= 1."""
    if not (0 <= rank < world) or n_total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_results(dist, ranks, phi, n_total, world, rank):
    """Gather per-rank (ranks [k, nt] int16, phi [k] float64) to rank 0, in global subproblem order.

    Blocks are padded to the largest shard, because `gather` needs equal shapes. Returns the assembled
    (ranks [n_total, nt], phi [n_total]) on rank 0, and (None, None) elsewhere.
    """
    import torch
    kmax = -(-n_total // world)
    nt = ranks.shape[1]
    k = ranks.shape[0]
    lo, hi = shard(n_total, world, rank)
    if k != hi - lo or phi.shape[0] != k:
        raise ValueError(f"rank {rank}: expected {hi - lo} results, got {k}")
    pr = torch.zeros((kmax, nt), dtype=ranks.dtype, device=ranks.device)
    pp = torch.zeros((kmax,), dtype=phi.dtype, device=phi.device)
    pr[:k] = ranks
    pp[:k] = phi
    if world == 1:
        return pr[:k], pp[:k]
    # RCCL/NCCL and gloo have no 16-bit integer type: the ranks travel as their bytes
    pb = pr.view(torch.uint8)
    gr = [torch.empty_like(pb) for _ in range(world)] if rank == 0 else None
    gp = [torch.empty_like(pp) for _ in range(world)] if rank == 0 else None
    dist.gather(pb, gr, dst=0)
    dist.gather(pp, gp, dst=0)
    if rank != 0:
        return None, None
    out_r, out_p = [], []
    for r in range(world):
        a, b = shard(n_total, world, r)
        out_r.append(gr[r].view(ranks.dtype)[: b - a])
        out_p.append(gp[r][: b - a])
    return torch.cat(out_r), torch.cat(out_p)


def level_ranks(u, nuval):
    """Controls u [k, nt, M] (level values) -> int16 level ranks [k, nt] (row of `nuval` [L, M])."""
    import torch
    k, nt, M = u.shape
    eq = (u.reshape(k * nt, 1, M) == nuval.reshape(1, *nuval.shape)).all(dim=2)
    if not bool(eq.any(dim=1).all()):
        raise ValueError("a control is not an admissible level tuple")
    return eq.int().argmax(dim=1).to(torch.int16).reshape(k, nt)
