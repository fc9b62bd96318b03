"""The frame-parallel RMSF pipeline of RMSF.py, on HIP kernels.

Per rank (one process per GPU):
  align=None      Welford over the block                    (rms.RMSF.run)
  align="frame0"  superpose every frame on frame ``ref_frame``, then Welford
  align="average" RMSF.py exactly: sweep 1 superposes on frame ``ref_frame``
                  and sums (RMSF.py:89-105); all-reduce + divide gives the
                  average structure (RMSF.py:107-111); sweep 2 superposes on
                  the centred average and runs Welford (RMSF.py:113-140).
then the cross-rank Chan merge (RMSF.py:141-143: one all-reduce of moments
about a shift every rank holds) and the finalise (RMSF.py:145-146).  Every
launch is asynchronous on the current stream; the only host synchronisation
is the final copy of the result.
"""
from __future__ import annotations

import contextlib
import os
from collections import defaultdict
from dataclasses import dataclass, field

import numpy as np
import torch

from . import parallel
from ._lib import (RMSF_MAX_SPLIT_FRAMES, RMSF_MODE_SUM, RMSF_MODE_WELFORD, RMSF_REFINFO_DOUBLES, RMSF_XFORM_DOUBLES,
                   RmsfEmptyError)
from .engine import Engine
from .sources import Batch, DeviceSource, FrameList, _scattered

ALIGN_MODES = (None, "frame0", "average")


class KernelTimer:
    """HIP-event spans recorded on the launching (current) stream around the
    ABI calls of the pipeline -- used by bench.py for the per-kernel roofline.
    Each span also records the atom-frames its launch processed, so a rate
    is sum(work) / sum(time) over launches of any size."""

    def __init__(self):
        self.spans = defaultdict(list)

    @contextlib.contextmanager
    def span(self, name: str, atom_frames: int = 0):
        s = torch.cuda.current_stream()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        yield
        b.record(s)
        self.spans[name].append((a, b, int(atom_frames)))

    def clear(self) -> None:
        self.spans.clear()

    def ms(self, name: str) -> list[float]:
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b, _ in self.spans.get(name, [])]

    def totals(self, name: str) -> tuple[int, float, int]:
        """(launches, summed ms, summed atom-frames) of ``name``."""
        t = self.ms(name)
        return len(t), float(sum(t)), sum(af for _, _, af in self.spans.get(name, []))


_NULL = contextlib.nullcontext()


def _span(timer, name, atom_frames: int = 0):
    return timer.span(name, atom_frames) if timer is not None else _NULL


class Accumulator:
    """Running Welford (or f64 sum) over streamed batches, on device.

    Default (``n_splits=None``): the balanced grid -- one equal (lane chunk,
    frame) range per workgroup, partials in ``work``, folded in frame order
    into ``parts0[0]``/``parts1[0]`` (the running result) by
    ``rmsf_fold_balanced``.  With a fixed ``n_splits`` the split grid is used:
    ``parts0/parts1`` are [1 + S_max, 3*n_sel] f64, slots 1..S hold the
    batch's split partials, folded into slot 0 by the Chan-merge kernel (or
    the split-sum kernel)."""

    def __init__(self, eng: Engine, n_sel: int, mode: int, max_batch: int, aligned: bool,
                 n_splits: int | None = None, timer: KernelTimer | None = None):
        self.eng, self.n_sel, self.mode, self.aligned = eng, n_sel, mode, aligned
        self.timer = timer
        self.n_coord = 3 * n_sel
        self.fixed_splits = n_splits
        self.work = None
        if n_splits:
            # a requested split count is raised where a tile would exceed the limit
            self.s_max = max(n_splits, -(-max_batch // RMSF_MAX_SPLIT_FRAMES))
        else:
            self.s_max = 0
            # the bound grows with the batch, so size it for the largest one
            nbytes = eng.balanced_workspace_bytes(n_sel, max_batch)
            self.work = eng.empty(max(2, (nbytes + 7) // 8))
        # Slot 0 is the running result.  The balanced fold overwrites it on the
        # first batch (acc_n = 0), so it is zeroed only if it is read with no
        # frames folded in (an empty block); the split grid's Chan merge reads
        # it from the start.  Split slots are written before they are read.
        self.parts0 = eng.empty(1 + self.s_max, self.n_coord)
        self.parts1 = None
        if mode == RMSF_MODE_WELFORD:
            self.parts1 = eng.empty(1 + self.s_max, self.n_coord)
        self.n = 0
        self.packed = False
        self.finalized = False
        self._zeroed = False
        if n_splits:
            self._zero()

    def _zero(self) -> None:
        if not self._zeroed:
            self.parts0[0].zero_()
            if self.parts1 is not None:
                self.parts1[0].zero_()
            self._zeroed = True

    def add(self, b: Batch, xform: torch.Tensor | None = None, refinfo: torch.Tensor | None = None,
            pack=None, fin=None) -> None:
        """``pack`` = (shift, off3, t, pending broadcast or None[, slice
        width]): this is the rank's last batch before the cross-rank merge;
        on the balanced grid in WELFORD mode the fold also writes the merge's
        moments about the shift into ``t`` (one launch; ``self.packed`` tells
        the caller) -- in the reduce-scatter merge's atom-sliced layout when a
        slice width is given.
        ``fin`` = (rmsf, n_total): the last batch of an aligned single-rank
        sweep; the fold also finalises (RMSF.py:146, ``self.finalized``)."""
        eng = self.eng
        p1 = None if self.parts1 is None else self.parts1[0]
        if not self.fixed_splits:
            need = eng.balanced_workspace_bytes(self.n_sel, b.n_frames)
            if need > self.work.numel() * 8:  # the bound is not monotone in the batch size
                self.work = eng.empty((need + 7) // 8)
            with _span(self.timer, "accumulate", b.n_frames * self.n_sel):
                eng.accumulate_balanced(b.ptr, b.fstride, b.n_frames, self.n_sel, b.sel, xform, refinfo, self.mode,
                                        self.work, pstride=b.pstride)
            if pack is not None and self.mode == RMSF_MODE_WELFORD:
                shift, off3, t, work = pack[:4]
                sc = pack[4] if len(pack) > 4 else None
                if work is not None:
                    work.wait()  # the shift's broadcast ran beside the sweep
                if sc:
                    eng.fold_balanced_shift_sliced(self.work, self.n_coord, self.n, self.parts0[0], p1, shift, off3,
                                                   sc, t)
                else:
                    eng.fold_balanced_shift(self.work, self.n_coord, self.n, self.parts0[0], p1, shift, off3, t)
                self.packed = True
            elif fin is not None and self.mode == RMSF_MODE_WELFORD and self.aligned:
                eng.fold_balanced_finalize(self.work, self.n_coord, self.n, self.parts0[0], p1, fin[1], fin[0])
                self.finalized = True
            else:
                eng.fold_balanced(self.work, self.n_coord, self.mode, self.n, self.parts0[0], p1)
            self.n += b.n_frames
            return
        if b.pstride:
            raise ValueError("coordinate planes are read in place on the balanced grid only (n_splits=None)")
        s = max(self.fixed_splits, -(-b.n_frames // RMSF_MAX_SPLIT_FRAMES))
        with _span(self.timer, "accumulate", b.n_frames * self.n_sel):
            eng.accumulate(b.ptr, b.fstride, b.n_frames, self.n_sel, b.sel, xform, refinfo, self.mode, s,
                           self.parts0[1:], None if self.parts1 is None else self.parts1[1:])
        if self.mode == RMSF_MODE_WELFORD:
            counts = [self.n] + eng.split_counts(b.n_frames, s)
            eng.chan_merge(self.parts0, self.parts1, counts, self.n_coord, self.parts0[0], self.parts1[0])
        else:
            eng.sum_splits(self.parts0, 1 + s, self.n_coord, self.parts0[0])
        self.n += b.n_frames

    @property
    def result0(self) -> torch.Tensor:
        if self.n == 0:
            self._zero()
        return self.parts0[0]

    @property
    def result1(self) -> torch.Tensor:
        if self.n == 0:
            self._zero()
        return self.parts1[0]


class Superposer:
    """Per-frame COM + inner product + QCP for one batch (rmsf_superpose)."""

    def __init__(self, eng: Engine, n_sel: int, max_batch: int, masses: torch.Tensor | None,
                 timer: KernelTimer | None = None):
        self.eng, self.n_sel, self.masses, self.timer = eng, n_sel, masses, timer
        self.xform = eng.empty(max_batch, RMSF_XFORM_DOUBLES)
        nbytes = eng.workspace_bytes(n_sel, max_batch)
        self.work = eng.empty(max(1, (nbytes + 7) // 8))

    def run(self, b: Batch, ref: torch.Tensor, refinfo: torch.Tensor, dense_out: int | None = None,
            dense_stride: int = 0) -> torch.Tensor:
        xf = self.xform[: b.n_frames]
        need = self.eng.workspace_bytes(self.n_sel, b.n_frames)
        if need > self.work.numel() * 8:  # stats_plan's bytes are not monotone in the batch size
            self.work = self.eng.empty((need + 7) // 8)
        with _span(self.timer, "superpose", b.n_frames * self.n_sel):
            self.eng.superpose(b.ptr, b.fstride, b.n_frames, self.n_sel, b.sel, self.masses, ref, refinfo, xf,
                               self.work, pstride=b.pstride, dense_out=dense_out, dense_stride=dense_stride)
        return xf


# Compaction of gathered selections on the aligned path (round 6): a gathered
# row read costs every 128-B line holding a selected atom, so below these
# densities the first pass over each frame writes its selected rows out once
# (an exact copy) and the later passes read them dense (DESIGN section 4,
# "Sparse selections").  The copy's writes beside the gathered read cost
# more than their bytes, so one sweep (frame-0 alignment: one later pass)
# only gains below ~1 in 4.5 (C3 at 1 in 4 -2 %, 1 in 6 +11 %, 1 in 2 -28 %),
# RMSF.py's two sweeps (three later passes) at every density up to 1 in 2
# (+8 % there, +52 % at 1 in 4; profiles/r06_workloads/probe_density.txt).
COMPACT_MAX_DENSITY = 0.5           # two sweeps (align="average")
COMPACT_MAX_DENSITY_ONE_SWEEP = 0.2  # one sweep (align="frame0")


class _Compactor:
    """The dense [frames, pitch] copy (rows of n_sel x 3 floats, padded to
    16 B) of a gathered selection's rows,
    written by the covariance pass as it stages them
    (rmsf_superpose_compact) and read by the accumulate and, ``resident``
    (the whole block fits in half the free HBM), by every pass of a later
    sweep (RMSF.py:124) with no gather at all; otherwise per batch.  A dense
    batch shorter than the pipeline's would change the batching (and the
    fold's bits), so then it is not used (``usable``)."""

    max_bytes: int | None = None  # None: half the free HBM (tests set a small cap for the per-batch form)

    def __init__(self, eng: Engine, n_sel: int, n_local: int, max_batch: int):
        self.n_sel = n_sel
        # rows padded to 16 B: the copy is written as float4 (a fixed store
        # count per tile, rmsf_kernels.hip k_frame_stats DENSE 2) and the
        # dense passes stage it as float4 (VEC4); the pad is never read
        self.pitch = (3 * n_sel + 3) // 4 * 4
        row = 4 * self.pitch
        budget = self.max_bytes
        if budget is None:
            budget = torch.cuda.mem_get_info(eng.device)[0] // 2
        cap = max(1, budget // row)
        self.resident = n_local <= cap
        self.frames = n_local if self.resident else max(1, min(max_batch, cap))
        self.usable = self.resident or self.frames >= max_batch
        self.buf = None
        if self.usable:
            self.buf = torch.empty((max(1, self.frames), self.pitch), dtype=torch.float32, device=eng.device)
        self.filled = False

    def ptr(self, k: int) -> int:
        return self.buf.data_ptr() + 4 * self.pitch * k

    def dense(self, k: int, n: int) -> Batch:
        return Batch(self.ptr(k), self.pitch, n, None)

    def resident_batches(self, n_local: int, max_batch: int):
        for k in range(0, n_local, max_batch):
            yield self.dense(k, min(max_batch, n_local - k))


@dataclass
class PipelineResult:
    # None on the non-root ranks of a reduce-to-root merge (merge_root)
    rmsf: torch.Tensor | None     # f64 [n_sel]
    mean: torch.Tensor | None     # f64 [n_sel, 3]
    m2: torch.Tensor | None       # f64 [n_sel, 3]  (sum of squares, RMSF.py:120)
    n_frames: int                 # frames over all ranks
    n_local: int                  # frames of this rank's block
    block: tuple[int, int]
    average: torch.Tensor | None = None   # f64 [n_sel, 3] (align="average")
    rmsd: torch.Tensor | None = None      # f64 [n_local] last-sweep QCP rmsd
    # f64 [n_local, 16] per-frame transform records (R row-major 0..8, mobile
    # COM 9..11, rmsd 12) of the last sweep / of RMSF.py's first sweep
    transforms: torch.Tensor | None = None
    transforms_sweep1: torch.Tensor | None = None
    extras: dict = field(default_factory=dict)


# Below this many frames an aligned run takes the exact path by default.  One
# f32 rounding flip of an aligned coordinate (the frame-parallel sums round
# the rotation differently, RMSF.py:99-101) moves that atom's RMSF by
# |x_k - mean| ulp(x) (1 - 1/N) / (N RMSF) <= ulp(x) / sqrt(N), since
# |x_k - mean| <= sqrt(N) RMSF; with coordinates below 256 A (ulp <= 1.53e-5 A)
# that bound is under the north star's 1e-6 A from 234 frames.  Measured:
# 7 of 1,600 runs of 2-10 frames exceed 1e-6 A on the frame-parallel path
# (worst 2.98e-6 A), none on the exact one (profiles/r06_workloads/
# fuzz_fewframes_50seeds.txt); DESIGN section 5.
AUTO_EXACT_FRAMES = 256


def auto_exact_frames() -> int:
    """AUTO_EXACT_FRAMES, or the environment's RMSF_AUTO_EXACT_FRAMES (0 =
    never: the test suite's setting, so its many small aligned cases keep
    exercising the frame-parallel kernels they were written for)."""
    v = os.environ.get("RMSF_AUTO_EXACT_FRAMES")
    return AUTO_EXACT_FRAMES if v is None else int(v)


def auto_exact(align, n_frames: int, *, n_splits=None, merge_scatter: bool = False, merge_slabs=None) -> bool:
    """exact=None's choice: the sequential (bit-exact) path for aligned runs
    of fewer than AUTO_EXACT_FRAMES frames, where the frame-parallel path's
    rounding could exceed 1e-6 A; not where the caller asked for a
    frame-parallel-only form (split grid, scatter merge, atom slabs)."""
    return (align is not None and 0 < n_frames < auto_exact_frames() and not n_splits and not merge_scatter
            and merge_slabs in (None, 0, 1))


def _scattered_block(frames: FrameList, b0: int, b1: int, max_batch: int) -> bool:
    """The source reads this block as gathered compact batches already."""
    return _scattered(frames, b0, b1, max_batch)


def reference_from_frame(eng: Engine, source, frame: int, n_sel: int, masses, owner: int | None = None,
                         mass_total: float | None = None, after_centre=None):
    """RMSF.py:80-87: centred f64 reference of trajectory frame ``frame``.

    RMSF.py has every rank re-read that frame from disk.  Here, if every rank
    holds it (host / full-trajectory sources) each computes it locally;
    otherwise (sharded HBM-resident trajectories) the lowest rank holding it
    computes it and broadcasts 3*n_sel + 16 doubles.  ``mass_total`` given:
    the reference's own summation order (exact=True,
    rmsf_reference_setup_sequential; numpy's masses.sum()); ``after_centre``
    as Engine.reference_setup_seq takes it."""
    if mass_total is not None:
        def setup(b):
            _, r, i = eng.reference_setup_seq(n_sel, mass_total, frame_ptr=b.ptr, sel=b.sel, masses=masses,
                                              after_centre=after_centre)
            return r, i
    else:
        def setup(b):
            return eng.reference_setup(n_sel, frame_ptr=b.ptr, sel=b.sel, masses=masses)
    rank, size = parallel.world()
    if size > 1:
        if owner is None:
            have = bool(source.holds(frame))
            t = torch.tensor([rank if have else size, 0 if have else 1], dtype=torch.int64, device=eng.device)
            lo = t[:1].clone()
            missing = t[1:].clone()
            torch.distributed.all_reduce(lo, op=torch.distributed.ReduceOp.MIN)
            torch.distributed.all_reduce(missing, op=torch.distributed.ReduceOp.SUM)
            lo, missing = int(lo.item()), int(missing.item())
            if lo >= size:
                raise IndexError(f"reference frame {frame} is not held by any rank")
            owner = None if missing == 0 else lo
        if owner is not None:
            ref = eng.empty(n_sel, 3)
            info = eng.empty(RMSF_REFINFO_DOUBLES)
            if rank == owner:
                b = source.reference(frame, eng.stream)
                r, i = setup(b)
                b.done()
                ref.copy_(r)
                info.copy_(i)
            parallel.broadcast_(ref, owner)
            parallel.broadcast_(info[:16], owner)  # the record; the rest is setup scratch
            return ref, info
    b = source.reference(frame, eng.stream)
    r, i = setup(b)
    b.done()
    return r, i


def _frame_shift(eng: Engine, source, frames: FrameList, n_total: int, size: int, rank: int, raw: bool = False):
    """Frame 0 of the list, selected, as f32 on every rank: gathered by the
    rank whose RMSF.py:65-69 block starts with it and broadcast asynchronously
    (the broadcast runs beside the sweep; the merge waits for it).  ``raw``:
    as stored (coordinate planes read in place stay in plane order)."""
    from .sources import DeviceSource

    ref_of = source.raw_reference if raw else source.reference

    owner = next(r for r, (a, b) in enumerate(parallel.blocks(n_total, size)) if b > a)
    buf = torch.empty(3 * source.n_sel, dtype=torch.float32, device=eng.device)
    idx = eng.zero_index()
    if not isinstance(source, DeviceSource):  # staged / decoded on the launching stream
        if rank == owner:
            b = ref_of(frames[0], eng.stream)
            eng.gather_frames(b.ptr, b.fstride, idx, 1, source.n_sel, b.sel, buf)
            b.done()
        return buf, parallel.broadcast_async(buf, owner)
    # HBM-resident frames: gather and broadcast from a side stream, so the
    # owner's sweep is not queued behind them
    main = torch.cuda.current_stream(eng.device)
    side = eng.side_stream
    side.wait_stream(main)
    with torch.cuda.stream(side):
        if rank == owner:
            b = ref_of(frames[0], eng.stream)
            eng.gather_frames(b.ptr, b.fstride, idx, 1, source.n_sel, b.sel, buf)
            b.done()
        work = parallel.broadcast_async(buf, owner)
    buf.record_stream(side)
    return buf, work


# Auto merge slabs from 1M selected atoms, 2 of them: at C4's share (1M x
# 2,500 frames) the cut costs 45 us of device time (+1.0 %; 4 slabs +85 us,
# profiles/r03_workloads/merge_slabs_c4_share.txt) and lets half of the 48 MB
# all-reduce run beside the second slab's stream
SLAB_MIN_ATOMS = 1_000_000
SLABS_AUTO = 2


def _slab_bounds(n_chunks: int, k: int) -> list[tuple[int, int]]:
    """k atom slabs of the flat plan's chunks, cut at multiples of 3 chunks
    (3 x 1024 coordinates = whole atoms)."""
    cuts = sorted({min(n_chunks, max(0, 3 * round(i * n_chunks / k / 3))) for i in range(1, k)} - {0, n_chunks})
    b = [0] + cuts + [n_chunks]
    return list(zip(b[:-1], b[1:]))


def _slab_sweep(eng: Engine, acc: "Accumulator", b: Batch, slabs: list, shift, off3, shift_work, timer,
                root: int | None = None):
    """The final Welford sweep of one resident batch in atom slabs (N > 1):
    slab k's accumulate + fold (which packs its [T1 | T2]) and the start of
    its all-reduce, then slab k+1 streams while that all-reduce runs.
    Every coordinate's partials, segments and fold are the whole launch's
    (rmsf_accumulate_balanced_slab), so the result is bit-identical to the
    unslabbed merge wherever the collective's summation order is (any 2
    ranks).  Returns [(t_k, j0, j1, work_k)]."""
    n_coord = acc.n_coord
    out = []
    for c0, c1 in slabs:
        j0, j1 = 1024 * c0, min(1024 * c1, n_coord)
        with _span(timer, "accumulate", b.n_frames * (j1 - j0) // 3):
            eng.accumulate_balanced_slab(b.ptr, b.fstride, b.n_frames, acc.n_sel, c0, c1, acc.work)
        if shift_work is not None:
            shift_work.wait()  # the shift's broadcast ran beside the first slab
            shift_work = None
        t = torch.empty(2 * (j1 - j0), dtype=torch.float64, device=eng.device)
        eng.fold_balanced_shift_slab(acc.work, n_coord, acc.n, acc.parts0[0], acc.parts1[0], shift, off3, t, c0, c1)
        work = parallel.allreduce_sum_async(t) if root is None else parallel.reduce_sum_async(t, root)
        out.append((t, j0, j1, work))
    acc.n += b.n_frames
    return out


def _rows_from_planes(eng: Engine, mean, m2, n_sel: int, n_total: int):
    """Plane-order statistics (coordinate planes read in place) to (atom, xyz)
    order, and the RMSF of RMSF.py:146 from them."""
    mean, m2 = eng.planes_to_rows(mean, n_sel), eng.planes_to_rows(m2, n_sel)
    rmsf = eng.empty(n_sel)
    eng.finalize(m2, n_sel, n_total, rmsf)
    return mean, m2, rmsf


def run_pipeline(eng: Engine, source, frames: FrameList, *, align=None, masses=None, ref_frame: int = 0,
                 max_batch: int | None = None, n_splits: int | None = None, collect_rmsd: bool = False,
                 ref_owner: int | None = None, block: tuple[int, int] | None = None,
                 timer: KernelTimer | None = None, collect_transforms: bool = False,
                 merge_slabs: int | None = None, merge_root: int | None = None,
                 merge_scatter: bool = False, exact: bool | None = None, merge_order: str = "mpi4py",
                 compact: bool | None = None) -> PipelineResult:
    """``merge_slabs`` (N > 1, no alignment, HBM-resident block in one batch,
    flat chunk-aligned plan): cut the final sweep into that many atom slabs
    so each slab's cross-rank all-reduce overlaps the next slab's stream;
    None = SLABS_AUTO from SLAB_MIN_ATOMS selected atoms, 0/1 = off.
    ``merge_root`` (N > 1): the final merge is a reduce to that rank, as
    RMSF.py:143's ``comm.reduce(root=0)``; the other ranks' results are None
    (rmsf, mean, m2), like RMSF.py's non-root ranks.
    ``merge_scatter`` (N > 1): the merge as a reduce-scatter by atom slices
    (parallel.global_chan_scatter): each rank finishes its slice and only
    the RMSF is gathered to ``merge_root`` (default 0); ``mean``/``m2`` are
    None and each rank's slice of them is in ``extras`` ("atom_slice",
    "slice_mean", "slice_m2").
    ``exact``: RMSF.py with the reference's own arithmetic and summation
    orders -- align=None: RMSF.py:120-146, each rank's block through the
    sequential Welford (rmsf_welford_sequential), ~1.1-1.15x the balanced
    path's time; aligned: RMSF.py:80-146, every per-frame COM / inner product atom by
    atom (rmsf_superpose_sequential), the sweep-1 sum and Welford frame by
    frame (rmsf_accumulate_sequential), the Allreduce of RMSF.py:110 in rank
    order and the references of RMSF.py:84-85 / 117-118 in order
    (rmsf_reference_setup_sequential).  The ranks are reduced by
    second_order_moments in RMSF.py:143's comm.reduce order (``merge_order``:
    "mpi4py", mpi4py's default binomial tree, or "rank";
    parallel.global_chan_exact), then RMSF.py:146: results bit-identical to
    RMSF.py's (on the restated upstream orders).
    ``exact=None`` (default): exact for an aligned run of fewer than
    AUTO_EXACT_FRAMES frames (auto_exact), the frame-parallel path otherwise.
    ``compact`` (aligned runs over a gathered selection of HBM-resident
    rows): the first pass writes the selected rows out dense and the later
    passes read them (_Compactor); None = below COMPACT_MAX_DENSITY (two
    sweeps) or COMPACT_MAX_DENSITY_ONE_SWEEP (one) selected atoms per frame
    atom.  Same bits either way."""
    if align not in ALIGN_MODES:
        raise ValueError(f"align must be one of {ALIGN_MODES}, got {align!r}")
    if exact is None:
        exact = auto_exact(align, len(frames), n_splits=n_splits, merge_scatter=merge_scatter,
                           merge_slabs=merge_slabs)
    if exact:
        if n_splits or merge_scatter or merge_slabs not in (None, 0, 1):
            raise ValueError("exact=True runs the sequential kernels: no n_splits, merge_scatter or merge_slabs")
        if align is None and (collect_rmsd or collect_transforms):
            raise ValueError("collect_rmsd / collect_transforms need an aligned run")
        return _run_exact(eng, source, frames, max_batch, block, timer, merge_root, merge_order, align=align,
                          masses=masses, ref_frame=ref_frame, ref_owner=ref_owner, collect_rmsd=collect_rmsd,
                          collect_transforms=collect_transforms)
    rank, size = parallel.world()
    n_total = len(frames)
    if n_total == 0:
        raise RmsfEmptyError(-4, "RMSF.run", "no frames selected")
    if merge_root is not None and not 0 <= merge_root < size:
        raise ValueError(f"merge_root {merge_root} is not a rank of this {size}-rank group")
    root = merge_root if size > 1 else None
    scatter = bool(merge_scatter) and size > 1
    if scatter and root is None:
        root = 0
    std = parallel.blocks(n_total, size)[rank]
    if block is not None and size > 1 and tuple(block) != std:
        # the merge's shift frame (and RMSF.py's decomposition) is defined by
        # the RMSF.py:65-69 blocks: every rank must run its own
        raise ValueError(f"rank {rank}: block {tuple(block)} is not the RMSF.py:65-69 block {std}")
    b0, b1 = block if block is not None else std
    n_local = b1 - b0
    n_sel = source.n_sel
    if max_batch is None:
        max_batch = max(1, n_local)
    max_batch = max(1, min(max_batch, max(1, n_local)))
    m_dev = None
    if masses is not None:
        m_dev = (masses.dev if isinstance(masses, UploadedMasses)
                 else torch.as_tensor(np.ascontiguousarray(masses, dtype=np.float64)).to(eng.device))
        if m_dev.numel() != n_sel:
            raise ValueError("masses must have one entry per selected atom")
    aligned = align is not None
    # coordinate planes read in place by the unaligned accumulate: statistics
    # in plane order, permuted to (atom, xyz) at the end
    planes = not aligned and not n_splits and bool(getattr(source, "native_planes", False))
    if scatter and planes:
        raise ValueError("merge_scatter: the statistics of coordinate planes read in place are in plane order, "
                         "not atom order; use merge_root")
    batches_of = source.raw_batches if planes else source.batches
    if not planes and not n_splits and isinstance(source, DeviceSource) and source.layout == "soa":
        batches_of = source.plane_batches_in_place  # the kernels' plane variants read HBM planes in place
    gathered = (aligned and not planes and isinstance(source, DeviceSource) and source.layout == "fac"
                and source.sel_dev is not None and not _scattered_block(frames, b0, b1, max_batch))
    if compact is None:
        dmax = COMPACT_MAX_DENSITY if align == "average" else COMPACT_MAX_DENSITY_ONE_SWEEP
        compact = gathered and n_sel <= dmax * source.n_atoms
    cmp = _Compactor(eng, n_sel, n_local, max_batch) if (compact and gathered and n_local) else None
    if cmp is not None and not cmp.usable:
        cmp = None
    sup = Superposer(eng, n_sel, max_batch, m_dev, timer) if aligned else None
    rmsd = eng.empty(n_local) if (aligned and collect_rmsd) else None
    keep = aligned and collect_transforms
    xf_last = eng.empty(n_local, RMSF_XFORM_DOUBLES) if keep else None
    xf_first = eng.empty(n_local, RMSF_XFORM_DOUBLES) if (keep and align == "average") else None
    average = None

    def sweep(acc: Accumulator, ref=None, info=None, xf_out=None, pack=None, slabs=None, fin=None):
        done, slabbed = 0, None
        if cmp is not None and cmp.resident and cmp.filled:   # a later sweep: the dense block, no gather
            batches = cmp.resident_batches(n_local, max_batch)
        else:
            batches = batches_of(frames, b0, b1, max_batch, eng.stream)
        for b in batches:
            xf, src_b = None, b
            if aligned:
                if cmp is not None and b.sel is not None:
                    k = done if cmp.resident else 0
                    xf = sup.run(b, ref, info, dense_out=cmp.ptr(k), dense_stride=cmp.pitch)
                    b = cmp.dense(k, b.n_frames)   # the accumulate reads the dense rows
                else:
                    xf = sup.run(b, ref, info)
                if rmsd is not None:
                    rmsd[done:done + b.n_frames].copy_(xf[:, 12])
                if xf_out is not None:
                    xf_out[done:done + b.n_frames].copy_(xf)
            last = done + b.n_frames == n_local
            # the slab kernels read each frame as 3n contiguous floats: rows,
            # or unpadded planes (never a plane stride wider than the atoms)
            if slabs and done == 0 and last and b.sel is None and xf is None and not b.pstride:
                n_chunks = eng.balanced_slab_chunks(b.ptr, b.fstride, b.n_frames, n_sel)
                if n_chunks >= 2 * 3:
                    shift_, off3_, _, work_ = pack[:4]
                    slabbed = _slab_sweep(eng, acc, b, _slab_bounds(n_chunks, slabs), shift_, off3_, work_, timer,
                                          root)
            if slabbed is None:
                acc.add(b, xf, info, pack if last else None, fin if last else None)
            done += b.n_frames
            src_b.done()
        if cmp is not None and cmp.resident:
            cmp.filled = True
        return slabbed

    if align == "average":
        ref0, info0 = reference_from_frame(eng, source, ref_frame, n_sel, m_dev, ref_owner)
        acc1 = Accumulator(eng, n_sel, RMSF_MODE_SUM, max_batch, True, n_splits, timer)
        if n_local:
            sweep(acc1, ref0, info0, xf_first)
        total = parallel.allreduce_sum_(acc1.result0)       # RMSF.py:110
        # RMSF.py:111 + 113-118: the average and the reference from it
        average, ref, info = eng.reference_setup_mean(total, float(n_total), n_sel, m_dev)
    elif align == "frame0":
        ref, info = reference_from_frame(eng, source, ref_frame, n_sel, m_dev, ref_owner)
    else:
        ref = info = None

    # The merge's shift (parallel.global_chan_shifted): something every rank
    # holds near the data -- the last sweep's reference structure, or (no
    # alignment) frame 0 of the list, broadcast by its owner while the sweep
    # streams.
    shift = off3 = shift_work = None
    if size > 1:
        if align == "average":
            shift = average
        elif align == "frame0":
            shift, off3 = ref, info[:3]
        else:
            shift, shift_work = _frame_shift(eng, source, frames, n_total, size, rank, raw=planes)

    acc = Accumulator(eng, n_sel, RMSF_MODE_WELFORD, max_batch, aligned, n_splits, timer)
    # N > 1: the last batch's fold also packs the merge's moments (one launch);
    # large selections in one resident batch run as overlapped atom slabs
    sc = 3 * -(-n_sel // size) if scatter else None   # the reduce-scatter's slice width (coordinates)
    t = (torch.empty(2 * sc * size if scatter else 6 * n_sel, dtype=torch.float64, device=eng.device)
         if size > 1 else None)
    k_slabs = merge_slabs if merge_slabs is not None else (SLABS_AUTO if n_sel >= SLAB_MIN_ATOMS else 0)
    slabs = k_slabs if (size > 1 and k_slabs > 1 and not aligned and not n_splits and not scatter) else None
    slabbed = None
    # one rank, aligned: the last fold also finalises (RMSF.py:146)
    rmsf_fin = eng.empty(n_sel) if (size == 1 and aligned) else None
    if n_local:
        slabbed = sweep(acc, ref, info, xf_last, (shift, off3, t, shift_work, sc) if size > 1 else None, slabs,
                        (rmsf_fin, n_total) if rmsf_fin is not None else None)
    if slabbed is not None:                                  # RMSF.py:141-143 + 146, slab by slab
        if root is not None and rank != root:
            with _span(timer, "merge"):                      # the exposed part: waits for the slabs' reduces
                for *_, work in slabbed:
                    if work is not None:
                        work.wait()
            return PipelineResult(rmsf=None, mean=None, m2=None, n_frames=n_total, n_local=n_local, block=(b0, b1),
                                  average=None, rmsd=rmsd, extras={"merge_slabs": len(slabbed), "merge_root": root})
        mean, m2, rmsf = eng.empty(3 * n_sel), eng.empty(3 * n_sel), eng.empty(n_sel)
        with _span(timer, "merge"):
            for t_k, j0, j1, work in slabbed:
                if work is not None:
                    work.wait()
                eng.chan_shift_finish(t_k, shift[j0:j1], off3, (j1 - j0) // 3, n_total, mean[j0:j1], m2[j0:j1],
                                      rmsf[j0 // 3:j1 // 3])
        if planes:
            mean, m2, rmsf = _rows_from_planes(eng, mean, m2, n_sel, n_total)
        return PipelineResult(rmsf=rmsf, mean=mean.view(n_sel, 3), m2=m2.view(n_sel, 3), n_frames=n_total,
                              n_local=n_local, block=(b0, b1), average=None, rmsd=rmsd,
                              extras={"merge_slabs": len(slabbed), "merge_root": root})
    if scatter:                                              # RMSF.py:141-143 + 146 by atom slices
        with _span(timer, "merge"):
            rmsf, mean_s, m2_s, (a0, a1) = parallel.global_chan_scatter(
                eng, acc.result0, acc.result1, acc.n, n_total, shift, off3, None if acc.packed else shift_work,
                packed=t if acc.packed else None, slice_coords=sc, root=root)
        return PipelineResult(rmsf=rmsf, mean=None, m2=None, n_frames=n_total, n_local=n_local, block=(b0, b1),
                              average=None if average is None else average.view(n_sel, 3), rmsd=rmsd,
                              transforms=xf_last, transforms_sweep1=xf_first,
                              extras={"merge_root": root, "merge": "scatter", "atom_slice": (a0, a1),
                                      "slice_mean": mean_s.view(-1, 3), "slice_m2": m2_s.view(-1, 3)})
    if size > 1:                                             # RMSF.py:141-143 + 146: one all-reduce
        # "merge" span: from the packed moments to the finished result on the
        # launching stream -- the collective (incl. waiting for the slowest
        # rank) and the unpack/finalise
        with _span(timer, "merge"):
            mean, m2, rmsf = parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, n_total,
                                                          shift, off3, None if acc.packed else shift_work,
                                                          packed=t if acc.packed else None, root=root)
        if planes and rmsf is not None:
            mean, m2, rmsf = _rows_from_planes(eng, mean, m2, n_sel, n_total)
        if rmsf is None:                                     # a non-root rank of the reduce
            return PipelineResult(rmsf=None, mean=None, m2=None, n_frames=n_total, n_local=n_local,
                                  block=(b0, b1), average=None if average is None else average.view(n_sel, 3),
                                  rmsd=rmsd, transforms=xf_last, transforms_sweep1=xf_first,
                                  extras={"merge_root": root})
    elif planes:
        mean, m2, rmsf = _rows_from_planes(eng, acc.result0, acc.result1, n_sel, n_total)
    else:
        mean, m2 = acc.result0, acc.result1
        if acc.finalized:                                    # RMSF.py:146, in the last fold
            rmsf = rmsf_fin
        else:
            rmsf = eng.empty(n_sel)
            eng.finalize(m2, n_sel, n_total, rmsf)           # RMSF.py:146
    return PipelineResult(rmsf=rmsf, mean=mean.view(n_sel, 3), m2=m2.view(n_sel, 3), n_frames=n_total,
                          n_local=n_local, block=(b0, b1),
                          average=None if average is None else average.view(n_sel, 3), rmsd=rmsd,
                          transforms=xf_last, transforms_sweep1=xf_first)


EXACT_OVERLAP_MIN_ATOMS = 16384


def _run_exact(eng: Engine, source, frames: FrameList, max_batch, block, timer, merge_root,
               merge_order: str = "mpi4py", *, align=None, masses=None, ref_frame: int = 0,
               ref_owner: int | None = None, collect_rmsd: bool = False,
               collect_transforms: bool = False) -> PipelineResult:
    """run_pipeline(exact=True): RMSF.py bit for bit (see there)."""
    rank, size = parallel.world()
    n_total = len(frames)
    if n_total == 0:
        raise RmsfEmptyError(-4, "RMSF.run", "no frames selected")
    if merge_root is not None and not 0 <= merge_root < size:
        raise ValueError(f"merge_root {merge_root} is not a rank of this {size}-rank group")
    root = merge_root if size > 1 else None
    blocks = parallel.blocks(n_total, size)
    if block is not None and size > 1 and tuple(block) != blocks[rank]:
        raise ValueError(f"rank {rank}: block {tuple(block)} is not the RMSF.py:65-69 block {blocks[rank]}")
    b0, b1 = block if block is not None else blocks[rank]
    n_local = b1 - b0
    n_sel = source.n_sel
    max_batch = max(1, min(max_batch or max(1, n_local), max(1, n_local)))
    aligned = align is not None
    m_dev, mass_total = None, float(n_sel)
    if masses is not None:
        m_np = masses.host if isinstance(masses, UploadedMasses) else np.ascontiguousarray(masses, dtype=np.float64)
        if m_np.size != n_sel:
            raise ValueError("masses must have one entry per selected atom")
        # AtomGroup.center_of_mass divides by weights.sum(): numpy's own
        # (pairwise) sum of the f64 masses -- one host scalar
        mass_total = float(m_np.sum())
        m_dev = masses.dev if isinstance(masses, UploadedMasses) else torch.as_tensor(m_np).to(eng.device)
    xf = eng.empty(max_batch, RMSF_XFORM_DOUBLES) if aligned else None
    rmsd = eng.empty(n_local) if (aligned and collect_rmsd) else None
    xf_last = eng.empty(n_local, RMSF_XFORM_DOUBLES) if (aligned and collect_transforms) else None
    xf_first = eng.empty(n_local, RMSF_XFORM_DOUBLES) if (collect_transforms and align == "average") else None

    # The frames' COM chains need no reference, so one process runs the
    # reference's chains (rmsf_reference_setup_sequential) on a side stream
    # beside the first batch's COM chains, and the reference's sums beside
    # its InnerProduct (which needs only the centred reference; the QCP needs
    # the sums' G2): 2 serial chain phases per sweep, not 4.  (With ranks the
    # reference may come from a collective, and a host source stages its
    # frames on the current stream; those keep one stream.)  ``pending`` =
    # the side stream's two events (reference centred, record complete) the
    # first batch's InnerProduct and QCP wait for.
    # Below EXACT_OVERLAP_MIN_ATOMS a chain phase is microseconds and the
    # fork/join costs more than it saves.  The side stream is the engine's,
    # made once (creating a stream per run cost milliseconds).
    from .sources import DeviceSource
    overlap = aligned and size == 1 and isinstance(source, DeviceSource) and n_sel >= EXACT_OVERLAP_MIN_ATOMS
    main = torch.cuda.current_stream(eng.device)
    side = None
    if overlap:
        side = getattr(eng, "_exact_side_stream", None)
        if side is None:
            side = eng._exact_side_stream = torch.cuda.Stream(eng.device)

    def on_side(fn):
        side.wait_stream(main)
        centred = torch.cuda.Event()
        with torch.cuda.stream(side):
            out = fn(lambda: centred.record(side))
        done = torch.cuda.Event()
        done.record(side)
        for t in out if isinstance(out, tuple) else (out,):
            if isinstance(t, torch.Tensor):
                t.record_stream(main)
        return out, (centred, done)

    def sweep(mode, acc0, acc1, ref=None, info=None, xf_out=None, pending=None):
        work, k = None, 0
        for b in source.batches(frames, b0, b1, max_batch, eng.stream):  # rows: (frame, atom, xyz)
            if b.pstride:
                raise ValueError("exact=True reads (frame, atom, xyz) rows; this source handed over coordinate planes")
            x = None
            if aligned:
                x = xf[:b.n_frames]
                with _span(timer, "superpose", b.n_frames * n_sel):
                    if pending is None:
                        eng.superpose_seq(b.ptr, b.fstride, b.n_frames, n_sel, b.sel, m_dev, mass_total, ref, info,
                                          x)
                    else:
                        eng.frame_com_seq(b.ptr, b.fstride, b.n_frames, n_sel, b.sel, m_dev, mass_total, x)
                        main.wait_event(pending[0])
                        eng.inner_product_seq(b.ptr, b.fstride, b.n_frames, n_sel, b.sel, ref, x)
                        main.wait_event(pending[1])
                        pending = None
                        eng.superpose_seq_qcp(b.n_frames, n_sel, info, x)
                if rmsd is not None:
                    rmsd[k:k + b.n_frames].copy_(x[:, 12])
                if xf_out is not None:
                    xf_out[k:k + b.n_frames].copy_(x)
            with _span(timer, "accumulate", b.n_frames * n_sel):
                if aligned:
                    work = eng.accumulate_seq(b.ptr, b.fstride, b.n_frames, n_sel, b.sel, x, info, mode, k, acc0,
                                              acc1, work)
                else:
                    work = eng.welford_sequential(b.ptr, b.fstride, b.n_frames, n_sel, b.sel, k, acc0, acc1, work)
            k += b.n_frames
            b.done()

    ref = info = average = pending = None
    if aligned:   # RMSF.py:80-87
        def ref_frame_setup(after_centre=None):
            return reference_from_frame(eng, source, ref_frame, n_sel, m_dev, ref_owner, mass_total=mass_total,
                                        after_centre=after_centre)
        if overlap:
            (ref, info), pending = on_side(ref_frame_setup)
        else:
            ref, info = ref_frame_setup()
    if align == "average":
        total = eng.zeros(3 * n_sel)                            # RMSF.py:89, selection rows
        if n_local:
            sweep(RMSF_MODE_SUM, total, None, ref, info, xf_first, pending)   # RMSF.py:91-103
        elif pending is not None:
            main.wait_event(pending[1])
        pending = None
        parallel.allreduce_sum_ordered_(eng, total)             # RMSF.py:110, rank order

        def ref_avg_setup(after_centre=None):                   # RMSF.py:111 + 113-118
            return eng.reference_setup_seq(n_sel, mass_total, total=total, n_frames=float(n_total), masses=m_dev,
                                           after_centre=after_centre)
        if overlap:
            (average, ref, info), pending = on_side(ref_avg_setup)
        else:
            average, ref, info = ref_avg_setup()
    mean, ss = eng.zeros(3 * n_sel), eng.zeros(3 * n_sel)       # RMSF.py:120-121
    if n_local:
        sweep(RMSF_MODE_WELFORD, mean, ss, ref, info, xf_last, pending)  # RMSF.py:123-138
    elif pending is not None:
        main.wait_event(pending[1])
    if size > 1:                                                # RMSF.py:141-143, comm.reduce's order
        with _span(timer, "merge"):
            mean, ss = parallel.global_chan_exact(eng, mean, ss, [e - s for s, e in blocks], root, merge_order)
    rmsf = None
    if mean is not None:
        rmsf = eng.empty(n_sel)
        eng.finalize(ss, n_sel, n_total, rmsf)                  # RMSF.py:146
    return PipelineResult(rmsf=rmsf, mean=None if mean is None else mean.view(n_sel, 3),
                          m2=None if ss is None else ss.view(n_sel, 3), n_frames=n_total, n_local=n_local,
                          block=(b0, b1), average=None if average is None else average.view(n_sel, 3), rmsd=rmsd,
                          transforms=xf_last, transforms_sweep1=xf_first,
                          extras={"exact": True, "merge_root": root, "merge_order": merge_order})


class UploadedMasses:
    """Masses already on the device, with their host copy (for the host
    scalar mass_total): CapturedPipeline uploads them before capture, since
    a host-to-device copy cannot be recorded into a graph."""

    def __init__(self, masses, device):
        self.host = np.ascontiguousarray(masses, dtype=np.float64)
        self.dev = torch.as_tensor(self.host).to(device)

    def __len__(self) -> int:
        return self.host.size


class CapturedPipeline:
    """The whole pipeline of ``run_pipeline`` recorded once into a hipGraph
    (``torch.cuda.CUDAGraph``) and replayed with no per-kernel host work.

    For latency-bound sizes (e.g. config C1: 214 atoms x 98 frames, ~15
    launches whose kernels run for microseconds) the eager path is bound by
    host launch overhead; replay removes it.  Every ABI entry point used here
    is asynchronous and performs no allocation or synchronisation, so the
    launch sequence is capture-safe.  Restrictions: single process, and an
    HBM-resident ``DeviceSource`` (host stagers synchronise on events).  The
    input frames may be overwritten in place between replays; ``result``
    tensors are rewritten by every replay."""

    def __init__(self, eng: Engine, source, frames: FrameList, **kw):
        from .sources import DeviceSource

        if parallel.world()[1] > 1:
            raise NotImplementedError("graph capture is single-process (the RCCL merge is not captured)")
        if not isinstance(source, DeviceSource):
            raise TypeError("only HBM-resident (DeviceSource) pipelines can be captured")
        if kw.get("timer") is not None:
            raise ValueError("a KernelTimer cannot be captured")
        dev = eng.device
        if kw.get("masses") is not None and not isinstance(kw["masses"], UploadedMasses):
            kw["masses"] = UploadedMasses(kw["masses"], dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up outside capture (allocator pools, lazy init)
            run_pipeline(eng, source, frames, **kw)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.result = run_pipeline(eng, source, frames, **kw)

    def replay(self) -> PipelineResult:
        self.graph.replay()
        return self.result
