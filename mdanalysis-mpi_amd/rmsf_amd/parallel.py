"""Multi-GPU plumbing: frame-block decomposition and the cross-rank merges.

Replaces the mpi4py layer of RMSF.py:
  * RMSF.py:59-72  rank/size + contiguous frame blocks   -> ``blocks()``
  * RMSF.py:107-111 Barrier + Allreduce(SUM) of positions -> ``allreduce_sum_``
  * RMSF.py:141-143 Barrier + pickle comm.reduce(second_order_moments)
        -> ``global_chan_shifted``: the k-way Chan merge as ONE all-reduce(SUM)
           of moments about a shift every rank holds (the pipeline's form;
           ``root=r``: a reduce to rank r, RMSF.py:143's own shape), or
           ``global_chan``: the same merge as two all-reduce(SUM) passes
           (mean, then deviations), or ``global_chan_scatter``: a
           reduce-scatter of the same moments by atom slices, each rank
           finishing its slice, and only the RMSF gathered to the root --
           over RCCL (torch.distributed "nccl" backend = RCCL on ROCm).

One process per GPU (torch.distributed.run); the frames shard with no data
path collective except these exchange steps.  The merges take an ``ops``
object for their element-wise steps: on the GPU that is the ``Engine`` (HIP
kernels); the CPU gloo tests pass the oracle's restatement.
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


def allreduce_sum_ordered_(ops, t: torch.Tensor) -> torch.Tensor:
    """RMSF.py:110's ``Allreduce(SUM)`` with the ranks' buffers added in rank
    order, ((s_0 + s_1) + s_2) + ..., identically on every rank (exact=True):
    every rank's buffer is all-gathered and ``ops.sum_splits`` (the device's
    k_sum_splits) adds them in that order.  Two ranks' sum is the same bits
    in any order (RMSF.py's ``mpirun -n 2``); from three ranks an MPI
    library picks its own order (MPICH: recursive doubling or
    reduce-scatter/allgather by message size -- upstream, not restated), so
    rank order is this build's definition there.  In place; no-op for one
    process."""
    _, size = world()
    if size > 1:
        n = t.numel()
        g = all_gather_(t.reshape(-1)).view(size, n)
        ops.sum_splits(g, size, n, t.reshape(-1))
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


def allreduce_sum_async(t: torch.Tensor):
    """Start an in-place SUM across ranks; returns the work (wait() orders
    the then-current stream after it), or None for a single process."""
    _, size = world()
    if size > 1:
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
    return None


def reduce_sum_async(t: torch.Tensor, root: int):
    """Start a SUM of ``t`` into rank ``root`` (RMSF.py:143's
    ``comm.reduce(..., root=0)``); returns the work, or None for a single
    process.  Only ``root``'s ``t`` holds the sum afterwards."""
    _, size = world()
    if size > 1:
        return dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, async_op=True)
    return None


def broadcast_async(t: torch.Tensor, src: int):
    """Start an in-place broadcast from ``src``; returns the work (wait() orders
    the then-current stream after it), or None for a single process."""
    _, size = world()
    if size > 1:
        return dist.broadcast(t, src=src, async_op=True)
    return None


def global_chan_shifted(ops, mean_k: torch.Tensor, m2_k: torch.Tensor, n_k: int, n_total: int, shift: torch.Tensor,
                        off3: torch.Tensor | None = None, shift_work=None, packed: torch.Tensor | None = None,
                        root: int | None = None):
    """The k-way Chan merge in ONE all-reduce: moments about a shift c that
    every rank already holds (c = shift + off3 per xyz: the sweep's reference
    structure, the sweep-1 average, or frame 0 broadcast during the sweep).

    T1 = sum_k n_k (mean_k - c),  T2 = sum_k [M2_k + n_k (mean_k - c)^2]
    mean = c + T1/n,  M2 = T2 - T1^2/n   (= Chan's k-way merge in exact
    arithmetic; c within the fluctuation of the data keeps it free of
    cancellation).  Returns (mean, M2, rmsf) -- the finalise of RMSF.py:146 is
    fused into the unpacking.  ``shift_work``: the pending broadcast that
    fills ``shift``, waited for here (it ran beside the sweep).  ``packed``:
    T1/T2 already written by the last fold (rmsf_fold_balanced_shift).
    ``root``: reduce to that rank only, as RMSF.py:143 does (half the
    collective's bytes of an all-reduce); the other ranks get
    (None, None, None)."""
    rank, size = world()
    if n_total <= 0:
        raise ZeroDivisionError("global_chan_shifted: no frames on any rank")
    n = mean_k.numel()
    if packed is not None:
        t = packed
    else:
        t = torch.empty(2 * n, dtype=mean_k.dtype, device=mean_k.device)
        if shift_work is not None:
            shift_work.wait()
        ops.chan_shift_pack(mean_k, m2_k, shift, off3, float(n_k), t)
    if size > 1:
        if root is None:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        else:
            dist.reduce(t, dst=root, op=dist.ReduceOp.SUM)
            if rank != root:
                return None, None, None
    mean, m2 = torch.empty_like(mean_k), torch.empty_like(m2_k)
    rmsf = torch.empty(n // 3, dtype=mean_k.dtype, device=mean_k.device)
    ops.chan_shift_finish(t, shift, off3, n // 3, n_total, mean, m2, rmsf)
    return mean, m2, rmsf


def _staged(t: torch.Tensor) -> bool:
    """gloo moves CUDA tensors through host memory for some collectives and
    not at all for others: stage those through the host ourselves (rehearsal
    transport only; RCCL takes device tensors directly)."""
    return t.is_cuda and dist.get_backend() == "gloo"


def reduce_scatter_sum_(out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
    """``out`` (rank r) = sum over ranks of ``inp``'s r-th of ``size`` equal
    chunks (RCCL reduce-scatter); ``out`` = ``inp`` for a single process."""
    _, size = world()
    if size == 1:
        out.copy_(inp[:out.numel()])
    elif _staged(inp):
        h = torch.empty(out.numel(), dtype=out.dtype)
        dist.reduce_scatter_tensor(h, inp.cpu())
        out.copy_(h)
    else:
        dist.reduce_scatter_tensor(out, inp)
    return out


def gather_(t: torch.Tensor, root: int):
    """Every rank's ``t`` (equal sizes) concatenated in rank order on
    ``root``; None on the other ranks."""
    rank, size = world()
    if size == 1:
        return t
    staged = _staged(t)
    src = t.cpu() if staged else t
    parts = [torch.empty_like(src) for _ in range(size)] if rank == root else None
    dist.gather(src, parts, dst=root)
    if rank != root:
        return None
    out = torch.cat(parts)
    return out.to(t.device) if staged else out


def all_gather_(t: torch.Tensor) -> torch.Tensor:
    """Every rank's ``t`` (equal sizes) concatenated in rank order, on every
    rank."""
    _, size = world()
    if size == 1:
        return t
    staged = _staged(t)
    src = t.cpu() if staged else t
    parts = [torch.empty_like(src) for _ in range(size)]
    dist.all_gather(parts, src)
    out = torch.cat(parts)
    return out.to(t.device) if staged else out


def _send(t: torch.Tensor, dst: int) -> None:
    dist.send(t.cpu() if _staged(t) else t, dst)


def _recv(like: torch.Tensor, src: int) -> torch.Tensor:
    if _staged(like):
        h = torch.empty(like.shape, dtype=like.dtype)
        dist.recv(h, src)
        return h.to(like.device)
    t = torch.empty_like(like)
    dist.recv(t, src)
    return t


MERGE_ORDERS = ("mpi4py", "rank")


def global_chan_exact(ops, mean_k: torch.Tensor, m2_k: torch.Tensor, counts: list[int], root: int | None = None,
                      order: str = "mpi4py"):
    """RMSF.py:141-143 with second_order_moments' own arithmetic (the
    device's k_chan_pair / k_chan_merge: RMSF.py:36-41 bit for bit), applied
    in the order RMSF.py:143's ``comm.reduce(S, root=0, op=...)`` applies it.
    ``counts`` = the ranks' frame counts (RMSF.py:65-69's blocks).

    ``order="mpi4py"`` (default): mpi4py's object reduce as it runs by default
    (``rc.fast_reduce``: PyMPI_reduce_p2p, upstream, unverified here) --
    point to point, a binomial tree: for mask = 1, 2, 4, ... a rank with the
    mask bit set sends its result (mean | M2) to ``rank & ~mask`` and stops;
    the others receive from ``rank | mask`` and compute op(result, received)
    on the device.  ``order="rank"``: mpi4py's naive reduce
    (``rc.fast_reduce = False``): every S gathered, folded in rank order.
    The two coincide up to 3 ranks and differ in the last bits from 4.

    ``root``: the result on that rank only (None elsewhere), as
    comm.reduce(root=...); None: on every rank.  Returns (mean, M2) or
    (None, None).  Merges of two empty states (T = 0, where RMSF.py:39
    raises) are skipped."""
    if order not in MERGE_ORDERS:
        raise ValueError(f"merge order must be one of {MERGE_ORDERS}, got {order!r}")
    rank, size = world()
    if size == 1:
        return mean_k, m2_k
    counts = [int(c) for c in counts]
    if len(counts) != size:
        raise ValueError("global_chan_exact: one frame count per rank expected")
    if sum(counts) == 0:
        raise ZeroDivisionError("global_chan_exact: no frames on any rank")
    n = mean_k.numel()
    if order == "rank":
        both = torch.cat([mean_k.reshape(-1), m2_k.reshape(-1)])
        g = all_gather_(both) if root is None else gather_(both, root)
        if g is None:
            return None, None
        g = g.view(size, 2, n)
        mean, m2 = torch.empty_like(mean_k), torch.empty_like(m2_k)
        ops.chan_merge(g[:, 0].contiguous(), g[:, 1].contiguous(), counts, n, mean, m2)
        return mean, m2
    # the binomial tree, each rank's `result` in its own buffer
    res = torch.cat([mean_k.reshape(-1), m2_k.reshape(-1)])
    have = counts[rank]
    mask = 1
    while mask < size:
        if rank & mask:
            _send(res, rank & ~mask)
            res = None
            break
        src = rank | mask
        if src < size:
            got = _recv(res, src)
            n_src = sum(counts[src:min(src + mask, size)])   # the frames of src's subtree
            if have + n_src > 0:
                ops.chan_merge_pair(res[:n], res[n:], have, got[:n], got[n:], n_src)
            have += n_src
        mask <<= 1
    # rank 0 holds comm.reduce's result: forward it to root (as mpi4py does),
    # or to every rank (root=None)
    if root is None:
        if res is None:
            res = torch.empty(2 * n, dtype=mean_k.dtype, device=mean_k.device)
        if _staged(res):
            h = res.cpu()
            dist.broadcast(h, 0)
            res = h.to(mean_k.device)
        else:
            dist.broadcast(res, 0)
    elif root != 0:
        if rank == 0:
            _send(res, root)
            res = None
        elif rank == root:
            res = _recv(torch.empty(2 * n, dtype=mean_k.dtype, device=mean_k.device), 0)
    if res is None or (root is not None and rank != root):
        return None, None
    return res[:n].clone(), res[n:].clone()


def global_chan_scatter(ops, mean_k: torch.Tensor, m2_k: torch.Tensor, n_k: int, n_total: int, shift: torch.Tensor,
                        off3: torch.Tensor | None = None, shift_work=None, packed: torch.Tensor | None = None,
                        slice_coords: int | None = None, root: int = 0):
    """The one-collective merge as a REDUCE-SCATTER by atom slices: rank r
    receives the summed T1/T2 of atoms [r p, (r+1) p) (p = ceil(n_sel/size)),
    finishes them (mean, M2 and RMSF.py:146 for its atoms), and only the RMSF
    (8 B per atom) is gathered to ``root`` -- RMSF.py:143's result on the
    root, with each rank's link carrying (size-1)/size of the moments plus
    the RMSF instead of the whole moments (reduce) or twice (all-reduce).
    ``packed``: the T1/T2 already written in the atom-sliced layout by the
    last fold (``slice_coords`` = 3 p).  Returns (rmsf on root else None,
    mean slice, M2 slice, (a0, a1)) -- the statistics stay sliced."""
    rank, size = world()
    if n_total <= 0:
        raise ZeroDivisionError("global_chan_scatter: no frames on any rank")
    n = mean_k.numel()
    n_sel = n // 3
    per = -(-n_sel // size)
    sc = 3 * per
    if slice_coords is not None and slice_coords != sc:
        raise ValueError(f"global_chan_scatter: packed with slice width {slice_coords}, expected {sc}")
    if packed is not None:
        t = packed
    else:
        t = torch.empty(2 * sc * size, dtype=mean_k.dtype, device=mean_k.device)
        if shift_work is not None:
            shift_work.wait()
        ops.chan_shift_pack_sliced(mean_k, m2_k, shift, off3, float(n_k), sc, t)
    zero_slice_padding(t, n, sc, size)
    out = torch.empty(2 * sc, dtype=t.dtype, device=t.device)
    reduce_scatter_sum_(out, t)
    a0, a1 = min(rank * per, n_sel), min((rank + 1) * per, n_sel)
    mean_s = torch.empty(3 * (a1 - a0), dtype=mean_k.dtype, device=mean_k.device)
    m2_s = torch.empty_like(mean_s)
    rmsf_s = torch.zeros(per, dtype=mean_k.dtype, device=mean_k.device)
    if a1 > a0:
        ops.chan_shift_finish_slice(out, sc, shift.reshape(-1)[3 * a0:], off3, a1 - a0, n_total, mean_s, m2_s,
                                    rmsf_s)
    full = gather_(rmsf_s, root)
    return (None if full is None else full[:n_sel]), mean_s, m2_s, (a0, a1)


def zero_slice_padding(t: torch.Tensor, n: int, sc: int, size: int) -> None:
    """Zero the never-written coordinates of the atom-sliced layout (past the
    n real ones, in the last slices), so the reduce-scatter sums zeros there."""
    for r in range(size):
        valid = max(0, min(sc, n - r * sc))
        if valid < sc:
            base = 2 * r * sc
            t[base + valid:base + sc].zero_()
            t[base + sc + valid:base + 2 * sc].zero_()


def barrier() -> None:
    _, size = world()
    if size > 1:
        dist.barrier()
