"""Batch sharding over ranks (SURVEY.md §8 e): partition + gather, world size 2 over gloo on the CPU.

The per-rank solver here is the CPU oracle (test double; on GPUs bench.py passes the libmioc context).
What is under test is the product's partition (`mioc.batch.shard`) and the rank-0 assembly
(`mioc.batch.gather_results`, the same code bench.py runs over RCCL).
"""
import os
import socket

import numpy as np
import pytest
import torch

from mioc.batch import gather_results, level_ranks, shard
from mioc.synth import CONFIGS, make_inputs

NT = 12


def test_shard_partition_is_contiguous_and_balanced():
    for n in range(0, 23):
        for world in range(1, 9):
            blocks = [shard(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard(4, 2, 2)


def _solve_block(lo, hi):
    """Restarts lo..hi-1 of config C5 (truncated nt), solved by the oracle: (ranks [k, nt] int16, phi [k])."""
    from oracle.oracle import Levels, OracleC, P_ONE
    cfg = CONFIGS["C5"]
    lt = cfg.levels()
    lv = Levels(lt.nu, [tuple(t) for t in lt.tuples])
    oc = OracleC()
    nuval = torch.tensor(lt.nuval, dtype=torch.float64)
    us, phis = [], []
    for k in range(lo, hi):
        _, df, uo = make_inputs(cfg, k=k, nt=NT, levels=lt)
        phi, U = oc.bellman(lv, df, uo, cfg.B, P_ONE, cfg.beta, cfg.dt)
        u, ps = oc.backtrack(lv, uo, phi, U, cfg.B, cfg.B)
        us.append(np.ascontiguousarray(u.T))
        phis.append(ps)
    u = torch.tensor(np.stack(us)) if us else torch.zeros((0, NT, lt.M), dtype=torch.float64)
    return level_ranks(u, nuval), torch.tensor(phis, dtype=torch.float64)


def _worker(rank, world, port, n_total, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard(n_total, world, rank)
        r, p = _solve_block(lo, hi)
        R, P = gather_results(dist, r, p, n_total, world, rank)
        if rank == 0:
            np.savez(out, ranks=R.numpy(), phi=P.numpy())
        else:
            assert R is None and P is None
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n_total", [5, 2])
def test_sharding_gloo_world2_matches_single_process(tmp_path, n_total):
    import torch.multiprocessing as mp
    out = str(tmp_path / "gathered.npz")
    mp.spawn(_worker, args=(2, _free_port(), n_total, out), nprocs=2, join=True)
    z = np.load(out)
    r1, p1 = _solve_block(0, n_total)
    assert z["ranks"].shape == (n_total, NT)
    assert np.array_equal(z["ranks"], r1.numpy())
    assert np.array_equal(z["phi"], p1.numpy())


def test_gather_single_rank_is_identity():
    r, p = _solve_block(0, 3)
    R, P = gather_results(None, r, p, 3, 1, 0)
    assert torch.equal(R, r) and torch.equal(P, p)
