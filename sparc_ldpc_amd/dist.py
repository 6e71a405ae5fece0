"""Multi-GPU Monte-Carlo plumbing: one process per GPU, reps
sharded by rank, one all-reduce of int64 error counters per round.

The data path has no collective: every rank decodes its own codewords on its
own device with the same operator (seed-0 ordering).  The only exchange is
the sum of ``[bit_errors, blocks, block_errors, iters]`` — 32 bytes — over
``torch.distributed`` (backend "nccl" = RCCL over xGMI on the MI355X node,
"gloo" on CPU for tests).  torch is plumbing here, not the product.
"""
from __future__ import annotations

import os

import numpy as np

__all__ = ["env_rank", "init", "allreduce_sum", "shard_seeds", "finalize"]


def env_rank():
    """(rank, world, local_rank) from the torchrun environment (defaults 0, 1, 0)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None):
    """Initialise torch.distributed when WORLD_SIZE > 1; returns (rank, world, local)."""
    rank, world, local = env_rank()
    if world > 1:
        import torch
        import torch.distributed as td
        if not td.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(local)
            td.init_process_group(backend)
    return rank, world, local


def allreduce_sum(arr: np.ndarray) -> np.ndarray:
    """Sum an int64 / float64 vector over all ranks (identity when not distributed)."""
    arr = np.ascontiguousarray(arr)
    try:
        import torch
        import torch.distributed as td
    except ImportError:
        return arr
    if not td.is_available() or not td.is_initialized() or td.get_world_size() == 1:
        return arr
    t = torch.from_numpy(arr.copy())
    if td.get_backend() == "nccl":
        t = t.cuda()
    td.all_reduce(t, op=td.ReduceOp.SUM)
    return t.cpu().numpy()


def shard_seeds(base: int, rnd: int, batch: int, rank: int, world: int):
    """Seeds of round `rnd` for `rank`: base + rnd*batch*world + rank + world*i.
    Disjoint across ranks and rounds; the union over ranks is contiguous."""
    start = base + rnd * batch * world
    return [start + rank + world * i for i in range(batch)]


def finalize():
    try:
        import torch.distributed as td
        if td.is_available() and td.is_initialized():
            td.destroy_process_group()
    except ImportError:
        pass
