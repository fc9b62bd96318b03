"""Multi-GPU plumbing: frame-block decomposition and the cross-rank merges.

Replaces the mpi4py layer of RMSF.py:
  * RMSF.py:59-72  rank/size + contiguous frame blocks   -> ``blocks()``
  * RMSF.py:107-111 Barrier + Allreduce(SUM) of positions -> ``allreduce_sum_``
  * RMSF.py:141-143 Barrier + pickle comm.reduce(second_order_moments)
        -> ``global_chan``: an exact k-way Chan merge as two all-reduce(SUM)
           passes over RCCL (torch.distributed "nccl" backend = RCCL on ROCm).

One process per GPU (torch.distributed.run); the frames shard with no data
path collective except these two exchange steps.  ``global_chan`` takes an
``ops`` object for its two element-wise steps: on the GPU that is the
``Engine`` (HIP kernels); the CPU gloo tests pass the oracle's restatement.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def blocks(n_frames: int, size: int) -> list[tuple[int, int]]:
    """RMSF.py:63-69: ``per = n // size``; ranks 0..size-2 get ``[i*per, (i+1)*per)``,
    the last rank ``[(size-1)*per, n)``.  (Pure Python mirror of rmsf_block_range.)"""
    if size < 1 or n_frames < 0:
        raise ValueError("blocks: size >= 1 and n_frames >= 0 required")
    per = n_frames // size
    out = [(i * per, (i + 1) * per) for i in range(size - 1)]
    out.append(((size - 1) * per, n_frames))
    return out


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    """In-place SUM across ranks (RMSF.py:110); no-op for a single process."""
    _, size = world()
    if size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def broadcast_(t: torch.Tensor, src: int) -> torch.Tensor:
    _, size = world()
    if size > 1:
        dist.broadcast(t, src=src)
    return t


def global_chan(ops, mean_k: torch.Tensor, m2_k: torch.Tensor, n_k: int, n_total: int):
    """Exact k-way Chan merge of per-rank (n_k, mean_k, M2_k) over all ranks.

    mean = sum_k (n_k/n) mean_k ;  M2 = sum_k [M2_k + n_k (mean_k - mean)^2]
    This equals folding second_order_moments (RMSF.py:36-41) over the ranks in
    exact arithmetic; empty ranks (n_k = 0, RMSF.py:39's ZeroDivisionError
    case) contribute zeros.  Returns new tensors (mean, M2) on every rank.
    """
    _, size = world()
    if size == 1:
        return mean_k, m2_k
    if n_total <= 0:
        raise ZeroDivisionError("global_chan: no frames on any rank")
    mean = torch.empty_like(mean_k)
    ops.chan_weight(mean_k, (n_k / n_total) if n_k else 0.0, mean)
    allreduce_sum_(mean)
    m2 = torch.empty_like(m2_k)
    ops.chan_deviation(mean_k, m2_k, mean, float(n_k), m2)
    allreduce_sum_(m2)
    return mean, m2


def barrier() -> None:
    _, size = world()
    if size > 1:
        dist.barrier()
