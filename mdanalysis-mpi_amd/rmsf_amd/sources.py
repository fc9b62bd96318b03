"""Frame sources: where device frame blocks come from.

RMSF.py reads frames with ``universe.trajectory[frame]`` (RMSF.py:92,124) and
re-decodes them on every sweep.  Here a source yields *device* batches of
frames (pointer, frame stride, count, selection) for a range of positions in
the frame list:

  * ``DeviceSource``  a float32 trajectory already resident in HBM (torch
    tensor [F, n_atoms, 3]); zero-copy, the selection is gathered in-kernel.
  * ``HostSource``    a host numpy float32 array, streamed through the pinned
    double-buffered ``Stager`` (C++ in csrc/stager.cpp).
  * ``XtcSource``     an XTC file: compressed records decompressed on the GPU
    (or on host threads into the stager).
  * ``DcdSource``     a DCD file: each batch's selected rows read from the
    memory-mapped file and staged.
  * ``AtomGroupSource`` an MDAnalysis AtomGroup (when MDAnalysis is present):
    ``ag.positions`` per Timestep, batched through the same stager.

Host sources can keep what they staged resident in HBM (``FrameCache``) so
that RMSF.py's second sweep does not cross PCIe again.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, Iterator

import numpy as np
import torch

from . import _lib
from ._lib import call


@dataclass
class Batch:
    ptr: int                      # device pointer of the first frame of the batch
    fstride: int                  # floats between consecutive frames
    n_frames: int
    sel: torch.Tensor | None      # int32 device selection (None = atoms 0..n_sel-1)
    release: Callable[[], None] | None = None
    pstride: int = 0              # > 0: frames stored as coordinate planes this many floats apart

    def done(self) -> None:
        if self.release is not None:
            self.release()
            self.release = None


class Stager:
    """ctypes handle on the C++ pinned multi-buffer stager (rmsf_stager_*)."""

    def __init__(self, n_atoms_frame: int, n_sel: int, sel, batch_frames: int, n_slots: int = 3,
                 n_threads: int = 4):
        self._h = ctypes.c_void_p()
        self._sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int32)
        sp = None if self._sel is None else self._sel.ctypes.data
        call("rmsf_stager_create", n_atoms_frame, n_sel, sp, batch_frames, n_slots, n_threads,
             ctypes.byref(self._h))
        self.batch_frames = batch_frames
        self.n_sel = n_sel

    def stage(self, host: np.ndarray, first: int, step: int, n: int, stream: int) -> tuple[int, int]:
        """Stage frames host[first], host[first+step], ... (n of them)."""
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        frame_floats = host.shape[1] * 3
        base = host.ctypes.data + first * frame_floats * 4
        call("rmsf_stager_stage", self._h, base, frame_floats * step, n, stream, ctypes.byref(slot),
             ctypes.byref(dptr))
        return slot.value, dptr.value

    def stage_ptrs(self, ptrs: np.ndarray, stream: int) -> tuple[int, int]:
        """Stage the frames at host addresses ``ptrs`` (uint64, one per frame)."""
        p = np.ascontiguousarray(ptrs, dtype=np.uint64)
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_stager_stage_ptrs", self._h, p.ctypes.data, p.size, stream, ctypes.byref(slot), ctypes.byref(dptr))
        return slot.value, dptr.value

    def stage_planes(self, ptrs: np.ndarray, plane_stride: int, stream: int) -> tuple[int, int]:
        """Stage the frames whose x planes start at host addresses ``ptrs``
        (uint64, one per frame; y and z ``plane_stride`` floats apart): the
        selection is interleaved into (frame, atom, xyz) rows on the host."""
        p = np.ascontiguousarray(ptrs, dtype=np.uint64)
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_stager_stage_planes", self._h, p.ctypes.data, int(plane_stride), p.size, stream,
             ctypes.byref(slot), ctypes.byref(dptr))
        return slot.value, dptr.value

    def stage_compact(self, buf: np.ndarray, n: int, stream: int) -> tuple[int, int]:
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_stager_stage", self._h, buf.ctypes.data, buf.shape[1] * 3, n, stream, ctypes.byref(slot),
             ctypes.byref(dptr))
        return slot.value, dptr.value

    def release(self, slot: int, stream: int) -> None:
        call("rmsf_stager_release", self._h, slot, stream)

    def synchronize(self) -> None:
        call("rmsf_stager_synchronize", self._h)

    def close(self) -> None:
        if self._h:
            call("rmsf_stager_destroy", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FrameList:
    """The frames of RMSF.run(): ``range(start, stop, step)`` or an explicit
    ``frames`` selection (indices or a boolean mask over the trajectory, as
    MDAnalysis' ``AnalysisBase.run(frames=...)`` takes).  An explicit list is
    taken in ascending order (duplicates kept): the statistics do not depend
    on the order beyond rounding.  Sources read it as ``runs()``: maximal
    arithmetic progressions of frames, each one strided batch."""

    def __init__(self, n_traj: int, start=None, stop=None, step=None, frames=None):
        self.idx = None
        if frames is not None:
            if start is not None or stop is not None or step is not None:
                raise ValueError("start/stop/step cannot be combined with frames")
            f = np.asarray(frames)
            if f.size == 0:
                f = f.astype(np.int64)
            elif f.dtype != bool and not np.issubdtype(f.dtype, np.integer):
                # AnalysisBase.run(frames=...) indexes with them: 1.7 is not a frame
                raise TypeError(f"frames must be integer indices or a boolean mask, got dtype {f.dtype}")
            if f.dtype == bool:
                if f.shape != (n_traj,):
                    raise ValueError(f"boolean frames must have one entry per frame ({n_traj})")
                f = np.flatnonzero(f)
            f = f.astype(np.int64).reshape(-1)
            if f.size and (f.min() < -n_traj or f.max() >= n_traj):
                raise IndexError(f"frame index out of range for {n_traj} frames")
            self.idx = np.sort(np.where(f < 0, f + n_traj, f), kind="stable")
            self.r = None
            return
        r = range(n_traj)[slice(start, stop, step)]
        if r.step < 0:  # reversed: the same frames ascending
            self.idx = np.array(r[::-1], dtype=np.int64)
            self.r = None
        else:
            self.r = r

    def __len__(self) -> int:
        return len(self.r) if self.r is not None else int(self.idx.size)

    def __getitem__(self, i: int) -> int:
        return self.r[i] if self.r is not None else int(self.idx[i])

    @property
    def start(self) -> int:
        return self[0]

    @property
    def step(self) -> int:
        if self.r is None:
            raise ValueError("an explicit frame list has no single step")
        return self.r.step

    def runs(self, b0: int, b1: int, max_n: int) -> Iterator[tuple[int, int, int]]:
        """(first frame, step >= 1, count) covering positions [b0, b1) in
        order, each at most ``max_n`` frames."""
        if self.r is not None:
            for i in range(b0, b1, max_n):
                yield self.r[i], self.r.step, min(max_n, b1 - i)
            return
        idx = self.idx
        i = b0
        while i < b1:
            st = int(idx[i + 1] - idx[i]) if i + 1 < b1 else 0
            j = i + 1
            if st > 0:
                while j < b1 and j - i < max_n and idx[j] - idx[j - 1] == st:
                    j += 1
            yield int(idx[i]), max(st, 1) if j > i + 1 else 1, j - i
            i = j


SCATTER_RUN = 8  # a frame list whose runs average fewer frames is read as gathered batches


def _scattered(frames: FrameList, b0: int, b1: int, nb: int) -> bool:
    """An explicit frame list whose block [b0, b1) is mostly short runs: read
    it as compact batches of up to ``nb`` frames (one gather / stage / decode
    each) instead of one batch -- and one set of kernel launches -- per run."""
    if frames.idx is None or b1 <= b0:
        return False
    return (b1 - b0) < SCATTER_RUN * sum(1 for _ in frames.runs(b0, b1, nb))


def _list_runs(rows: np.ndarray):
    """(first, step, n) runs of a sorted row list (arithmetic progressions)."""
    fl = FrameList(int(rows.max()) + 1 if rows.size else 0, frames=rows)
    return fl.runs(0, len(rows), max(1, len(rows)))


class _Gather:
    """A device scratch batch [nb, n_sel, 3] filled by rmsf_gather_frames from
    HBM-resident frames: one launch per batch of scattered frames.  Reused
    batch after batch -- the kernels that read it are queued on the same
    stream before the next gather."""

    def __init__(self, n_sel: int, nb: int, device):
        self.n_sel = n_sel
        self.buf = torch.empty((nb, n_sel, 3), dtype=torch.float32, device=device)

    def __call__(self, base_ptr: int, fstride: int, rows: np.ndarray, sel: torch.Tensor | None, stream: int) -> Batch:
        idx = torch.as_tensor(np.ascontiguousarray(rows, dtype=np.int64)).to(self.buf.device)
        call("rmsf_gather_frames", base_ptr, fstride, idx.data_ptr(), len(rows), self.n_sel,
             None if sel is None else sel.data_ptr(), self.buf.data_ptr(), stream)
        return Batch(self.buf.data_ptr(), 3 * self.n_sel, len(rows), None)


class _GatherPlanes(_Gather):
    """The same scratch batch filled by rmsf_gather_planes from HBM-resident
    coordinate planes (SoA frames)."""

    def __init__(self, n_sel: int, nb: int, device, plane_stride: int):
        super().__init__(n_sel, nb, device)
        self.plane_stride = plane_stride

    def __call__(self, base_ptr: int, fstride: int, rows: np.ndarray, sel: torch.Tensor | None, stream: int) -> Batch:
        idx = torch.as_tensor(np.ascontiguousarray(rows, dtype=np.int64)).to(self.buf.device)
        call("rmsf_gather_planes", base_ptr, fstride, self.plane_stride, idx.data_ptr(), len(rows), self.n_sel,
             None if sel is None else sel.data_ptr(), self.buf.data_ptr(), stream)
        return Batch(self.buf.data_ptr(), 3 * self.n_sel, len(rows), None)


def _gather_batch_frames(n_sel: int, nb: int) -> int:
    """Frames per gathered batch: the pipeline's batch, at most ~256 MB of scratch."""
    return max(1, min(nb, 65535, (256 << 20) // max(1, 12 * n_sel)))


class DeviceSource:
    """HBM-resident float32 trajectory [F_local, n_atoms, 3] holding global frames
    [offset, offset + F_local) of a trajectory with ``n_traj`` frames.

    ``layout="soa"``: the tensor is [F_local, 3, n_atoms] coordinate planes
    (atoms contiguous; frames and planes may be strided).  Each batch is
    gathered into a compact (frame, atom, xyz) scratch batch by
    rmsf_gather_planes first -- one extra read and write of the selected
    bytes, a convenience for frames that already live in HBM as planes."""

    layout = "fac"
    _planes = _ref_planes = None

    def __init__(self, traj: torch.Tensor, sel=None, offset: int = 0, n_traj: int | None = None,
                 layout: str = "fac"):
        if traj.dtype != torch.float32 or traj.device.type != "cuda":
            raise TypeError("DeviceSource needs a float32 tensor on a HIP device")
        if layout not in ("fac", "soa"):
            raise ValueError(f"layout must be 'fac' ([F, n_atoms, 3]) or 'soa' ([F, 3, n_atoms]), got {layout!r}")
        self.layout = layout
        if layout == "soa":
            if traj.dim() != 3 or traj.shape[1] != 3:
                raise ValueError("an SoA trajectory must be [n_frames, 3, n_atoms]")
            if traj.stride(2) != 1 or traj.stride(1) < traj.shape[2] or traj.stride(0) < 3 * traj.stride(1):
                raise ValueError("SoA frames must hold three contiguous, non-overlapping coordinate planes")
        else:
            if traj.dim() != 3 or traj.shape[2] != 3:
                raise ValueError("trajectory must be [n_frames, n_atoms, 3]")
            if traj.stride(2) != 1 or traj.stride(1) != 3:
                raise ValueError("trajectory frames must be contiguous [n_atoms, 3] rows")
        self.traj = traj
        self.n_atoms = traj.shape[2] if layout == "soa" else traj.shape[1]
        self.fstride = traj.stride(0)
        self.offset = offset
        self.n_traj = traj.shape[0] + offset if n_traj is None else n_traj
        self.sel_host = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.sel_host is not None:
            if self.sel_host.size and (self.sel_host.min() < 0 or self.sel_host.max() >= self.n_atoms):
                raise IndexError("selection index out of range")
        self.n_sel = self.n_atoms if sel is None else len(self.sel_host)
        self.sel_dev = None
        if self.sel_host is not None and not np.array_equal(self.sel_host, np.arange(self.n_sel)):
            self.sel_dev = torch.as_tensor(self.sel_host.astype(np.int32)).to(traj.device)

    def holds(self, frame: int) -> bool:
        return self.offset <= frame < self.offset + self.traj.shape[0]

    def _ptr(self, frame: int) -> int:
        if not self.holds(frame):
            raise IndexError(f"frame {frame} is not resident in this shard")
        return self.traj.data_ptr() + (frame - self.offset) * self.fstride * 4

    def reference(self, frame: int, stream: int) -> Batch:
        if self.layout == "soa":  # its own one-frame scratch: may run on a side stream beside a sweep's batches
            self._ptr(frame)
            if self._ref_planes is None:
                self._ref_planes = _GatherPlanes(self.n_sel, 1, self.traj.device, self.traj.stride(1))
            return self._ref_planes(self.traj.data_ptr(), self.fstride, np.array([frame - self.offset]),
                                    self.sel_dev, stream)
        return Batch(self._ptr(frame), self.fstride, 1, self.sel_dev)

    @property
    def n_rows(self) -> int:
        return self.traj.shape[0]

    def _plane_batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        """SoA: every batch (runs or a scattered list) gathered from the planes."""
        nb = max(1, min(max_frames, 65535, (512 << 20) // max(1, 12 * self.n_sel)))
        if self._planes is None or self._planes.buf.shape[0] < nb:
            self._planes = _GatherPlanes(self.n_sel, nb, self.traj.device, self.traj.stride(1))
        rows = frames.idx[b0:b1] if frames.idx is not None else np.arange(b0, b1, dtype=np.int64)
        if frames.idx is None and b1 > b0:
            rows = frames.r.start + frames.r.step * rows  # positions -> frame numbers
        for i in range(0, len(rows), nb):
            part = rows[i:i + nb]
            _check_run(self, int(part[0]), 1, 1, "HBM shard")
            _check_run(self, int(part[-1]), 1, 1, "HBM shard")
            yield self._planes(self.traj.data_ptr(), self.fstride, part - self.offset, self.sel_dev, stream)

    @property
    def native_planes(self) -> bool:
        """SoA frames the unaligned accumulate reads in place, as if they were
        rows (its statistics are per coordinate; they come out in plane
        order): three contiguous planes, no selection, float4-aligned."""
        return (self.layout == "soa" and self.sel_dev is None and self.traj.stride(1) == self.n_atoms
                and (3 * self.n_atoms) % 4 == 0 and self.fstride % 4 == 0 and self.traj.data_ptr() % 16 == 0)

    def raw_reference(self, frame: int, stream: int) -> Batch:
        """Frame ``frame`` as stored (planes stay planes)."""
        return Batch(self._ptr(frame), self.fstride, 1, self.sel_dev)

    def batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        if self.layout == "soa":
            yield from self._plane_batches(frames, b0, b1, max_frames, stream)
            return
        yield from self.raw_batches(frames, b0, b1, max_frames, stream)

    def plane_batches_in_place(self, frames: FrameList, b0: int, b1: int, max_frames: int,
                               stream: int) -> Iterator[Batch]:
        """SoA frames for the aligned kernels' plane variants
        (rmsf_superpose_planes, rmsf_accumulate_balanced_planes): runs read
        in place (``pstride`` set); a scattered list gathered into rows."""
        if _scattered(frames, b0, b1, max_frames):
            yield from self._plane_batches(frames, b0, b1, max_frames, stream)
            return
        for first, step, n in frames.runs(b0, b1, max_frames):
            _check_run(self, first, step, n, "HBM shard")
            yield Batch(self._ptr(first), self.fstride * step, n, self.sel_dev, pstride=self.traj.stride(1))

    def raw_batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        """Batches of the frames as stored: rows read in place (or gathered
        for a scattered list); for native_planes SoA frames, 3 n floats each."""
        if _scattered(frames, b0, b1, max_frames):
            nb = _gather_batch_frames(self.n_sel, max_frames)
            g = _Gather(self.n_sel, nb, self.traj.device)
            idx = frames.idx[b0:b1]
            for i in range(0, len(idx), nb):
                part = idx[i:i + nb]
                _check_run(self, int(part[0]), 1, 1, "HBM shard")
                _check_run(self, int(part[-1]), 1, 1, "HBM shard")
                yield g(self.traj.data_ptr(), self.fstride, part - self.offset, self.sel_dev, stream)
            return
        for first, step, n in frames.runs(b0, b1, max_frames):
            _check_run(self, first, step, n, "HBM shard")
            yield Batch(self._ptr(first), self.fstride * step, n, self.sel_dev)


def _check_run(src, first: int, step: int, n: int, what: str) -> None:
    """A run reads frames first, first+step, ..., first+step*(n-1): a sharded
    source must hold the last one too, or the kernels / the stager would read
    past the shard (runs are arithmetic, so first and last bound them all)."""
    for f in (first, first + step * (n - 1)):
        if not src.holds(f):
            lo = getattr(src, "offset", 0)
            raise IndexError(f"frame {f} is outside this {what} (frames [{lo}, {lo + src.n_rows})): the rank's "
                             "block of the frame list must lie inside the frames it holds")


class FrameCache:
    """Staged (selected) frames kept resident in HBM: RMSF.py reads every frame
    in both of its loops (RMSF.py:92,124), so the second sweep over a host
    source can read HBM instead of crossing PCIe (or MDAnalysis' reader)
    again.  Row r of the cache holds the source's row r, [n_sel, 3] float32;
    a batch whose rows are all present is served from the cache, otherwise
    it is staged and its rows are copied in (one strided device copy on the
    consumer stream, before the kernels that read them)."""

    def __init__(self, n_rows: int, n_sel: int, device=None):
        self.n_sel = n_sel
        self.buf = torch.empty((n_rows, n_sel, 3), dtype=torch.float32,
                               device=torch.cuda.current_device() if device is None else device)
        self.have = np.zeros(n_rows, dtype=bool)

    @staticmethod
    def fits(n_rows: int, n_sel: int) -> bool:
        """Cache only what takes at most half of the free device memory."""
        free, _ = torch.cuda.mem_get_info()
        return 12 * n_rows * n_sel <= free // 2

    def ptr(self, row: int) -> int:
        return self.buf.data_ptr() + 12 * self.n_sel * row

    def lookup(self, row: int, step: int, n: int) -> Batch | None:
        if self.have[row:row + step * (n - 1) + 1:step].all():
            return Batch(self.ptr(row), 3 * self.n_sel * step, n, None)
        return None

    def fill(self, row: int, step: int, n: int, src_ptr: int, stream: int) -> Batch:
        w = 12 * self.n_sel
        call("rmsf_memcpy2d_d2d", self.ptr(row), w * step, src_ptr, w, w, n, stream)
        self.have[row:row + step * (n - 1) + 1:step] = True
        return Batch(self.ptr(row), 3 * self.n_sel * step, n, None)

    def drop(self) -> None:
        self.have[:] = False

    def fill_rows(self, rows: np.ndarray, src_ptr: int, stream: int) -> None:
        """Copy a compact batch (frame k = rows[k]) into its rows, run by run."""
        w = 12 * self.n_sel
        k = 0
        for first, step, n in _list_runs(rows):
            call("rmsf_memcpy2d_d2d", self.ptr(first), w * step, src_ptr + w * k, w, w, n, stream)
            k += n
        self.have[rows] = True


def _cached_list(cache: FrameCache | None, gather, rows: np.ndarray, stream: int, stage) -> Batch:
    """Rows ``rows`` (a scattered list) of a host source as one compact batch:
    gathered from ``cache`` when all are resident; otherwise ``stage(rows)``
    -> compact Batch, copied into the cache when there is one."""
    if cache is not None and cache.have[rows].all():
        return gather(cache.buf.data_ptr(), 3 * cache.n_sel, rows, None, stream)
    b = stage(rows)
    if cache is not None:
        cache.fill_rows(rows, b.ptr, stream)
    return b


def _cached_stage(cache: FrameCache | None, row: int, step: int, n: int, stream: int, stage) -> Batch:
    """Rows [row, row+step, ...] of a host source: from ``cache`` when all are
    present; otherwise ``stage()`` -> Batch in a stager slot, whose rows are
    then copied into the cache (when there is one) and read from there."""
    if cache is not None:
        b = cache.lookup(row, step, n)
        if b is not None:
            return b
    b = stage()
    if cache is None:
        return b
    c = cache.fill(row, step, n, b.ptr, stream)
    c.release = b.release
    return c


class HostSource:
    """Host float32 array [F, n_atoms, 3] streamed through the pinned stager.
    Row r holds global frame ``offset + r`` of a trajectory of ``n_traj``
    frames (a rank's shard; default: the whole trajectory).  ``cache=True``
    keeps the staged frames resident in HBM for later sweeps (FrameCache;
    ignored when they would take more than half of the free device memory).
    A cached row is not re-read: call ``drop_cache()`` after changing the
    host array in place (``RMSF.run`` builds a fresh source per run).

    ``layout="soa"``: the array is [F, 3, n_atoms] -- each frame's x, y and
    z coordinate planes (structure of arrays; frames and planes may be
    strided, atoms contiguous).  The stager interleaves the selection into
    the (frame, atom, xyz) device batches on the host
    (rmsf_stager_stage_planes): same device frames, same results."""

    def __init__(self, traj: np.ndarray, sel=None, batch_frames: int | None = None, n_slots: int = 3,
                 n_threads: int = 4, offset: int = 0, n_traj: int | None = None, cache: bool = False,
                 layout: str = "fac"):
        if layout not in ("fac", "soa"):
            raise ValueError(f"layout must be 'fac' ([F, n_atoms, 3]) or 'soa' ([F, 3, n_atoms]), got {layout!r}")
        self.layout = layout
        if layout == "soa":
            traj = np.asarray(traj)
            if traj.ndim != 3 or traj.shape[1] != 3:
                raise ValueError("an SoA trajectory must be [n_frames, 3, n_atoms]")
            if traj.dtype != np.float32 or traj.strides[2] != 4 or traj.strides[0] % 4 or traj.strides[1] % 4 \
                    or traj.strides[0] < 0 or traj.strides[1] < 0:
                traj = np.ascontiguousarray(traj, dtype=np.float32)
        else:
            traj = np.ascontiguousarray(traj, dtype=np.float32)
            if traj.ndim != 3 or traj.shape[2] != 3:
                raise ValueError("trajectory must be [n_frames, n_atoms, 3]")
        self.traj = traj
        self.n_atoms = traj.shape[2] if layout == "soa" else traj.shape[1]
        self.offset = offset
        self.n_traj = traj.shape[0] + offset if n_traj is None else n_traj
        sel_arr = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if sel_arr is not None and sel_arr.size and (sel_arr.min() < 0 or sel_arr.max() >= self.n_atoms):
            raise IndexError("selection index out of range")
        self.n_sel = self.n_atoms if sel_arr is None else len(sel_arr)
        if batch_frames is None:  # ~64 MB per slot
            batch_frames = max(1, min(4096, (64 << 20) // max(1, 12 * self.n_sel)))
        self.batch_frames = batch_frames
        self.stager = Stager(self.n_atoms, self.n_sel, sel_arr, batch_frames, n_slots, n_threads)
        rows = traj.shape[0]
        self.cache = FrameCache(rows, self.n_sel) if cache and FrameCache.fits(rows, self.n_sel) else None

    def holds(self, frame: int) -> bool:
        return self.offset <= frame < self.offset + self.traj.shape[0]

    def drop_cache(self) -> None:
        """Forget the HBM-resident frames (the next sweep streams them again)."""
        if self.cache is not None:
            self.cache.drop()

    def _row(self, frame: int) -> int:
        if not self.holds(frame):
            raise IndexError(f"frame {frame} is not in this host shard")
        return frame - self.offset

    def _stage_rows(self, rows: np.ndarray, stream: int) -> Batch:
        """Host rows ``rows`` (any list) staged as one batch, one pointer per frame."""
        addr = (self.traj.ctypes.data + np.asarray(rows, dtype=np.int64) * self.traj.strides[0]).astype(np.uint64)
        if self.layout == "soa":
            slot, ptr = self.stager.stage_planes(addr, self.traj.strides[1] // 4, stream)
        else:
            slot, ptr = self.stager.stage_ptrs(addr, stream)
        return Batch(ptr, 3 * self.n_sel, len(addr), None, lambda: self.stager.release(slot, stream))

    def _stage(self, row: int, step: int, n: int, stream: int) -> Batch:
        def stage():
            if self.layout == "soa":
                return self._stage_rows(row + step * np.arange(n, dtype=np.int64), stream)
            slot, ptr = self.stager.stage(self.traj, row, step, n, stream)
            return Batch(ptr, 3 * self.n_sel, n, None, lambda: self.stager.release(slot, stream))

        return _cached_stage(self.cache, row, step, n, stream, stage)

    def reference(self, frame: int, stream: int) -> Batch:
        return self._stage(self._row(frame), 1, 1, stream)

    def batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        nb = min(max_frames, self.batch_frames)
        if _scattered(frames, b0, b1, nb):
            g = _Gather(self.n_sel, nb, self.cache.buf.device) if self.cache is not None else None
            idx = frames.idx[b0:b1]

            def stage(rows):
                return self._stage_rows(rows, stream)

            for i in range(0, len(idx), nb):
                part = idx[i:i + nb]
                _check_run(self, int(part[0]), 1, 1, "host shard")
                _check_run(self, int(part[-1]), 1, 1, "host shard")
                yield _cached_list(self.cache, g, part - self.offset, stream, stage)
            return
        for first, step, n in frames.runs(b0, b1, nb):
            _check_run(self, first, step, n, "host shard")
            yield self._stage(self._row(first), step, n, stream)

    @property
    def n_rows(self) -> int:
        return self.traj.shape[0]


class XtcDecoder:
    """ctypes handle on the pinned-slot GPU XTC decoder (rmsf_xtcdec_*)."""

    def __init__(self, xtc, batch_frames: int, n_slots: int = 3, n_threads: int = 8):
        self._h = ctypes.c_void_p()
        call("rmsf_xtcdec_create", xtc.handle, batch_frames, n_slots, n_threads, ctypes.byref(self._h))
        self.batch_frames, self.n_slots = batch_frames, n_slots

    def decode(self, first: int, n: int, step: int, stream: int) -> tuple[int, int]:
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_xtcdec_decode", self._h, first, n, step, stream, ctypes.byref(slot), ctypes.byref(dptr))
        return slot.value, dptr.value

    def decode_list(self, frames: np.ndarray, stream: int) -> tuple[int, int]:
        """Decode the frames ``frames`` (any list) into the next slot, in order."""
        f = np.ascontiguousarray(frames, dtype=np.int64)
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_xtcdec_decode_list", self._h, f.ctypes.data, f.size, stream, ctypes.byref(slot), ctypes.byref(dptr))
        return slot.value, dptr.value

    def decode_into(self, first: int, n: int, step: int, out_ptr: int, out_stride: int, stream: int) -> int:
        slot = ctypes.c_int()
        call("rmsf_xtcdec_decode_into", self._h, first, n, step, out_ptr, out_stride, stream, ctypes.byref(slot))
        return slot.value

    def release(self, slot: int, stream: int) -> None:
        call("rmsf_xtcdec_release", self._h, slot, stream)

    def synchronize(self) -> None:
        call("rmsf_xtcdec_synchronize", self._h)

    def close(self) -> None:
        if self._h:
            call("rmsf_xtcdec_destroy", self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class XtcSource:
    """GROMACS XTC file (the C5 path: an XTC-decoded trajectory streamed from
    the host).  ``decode="gpu"``: the compressed frame records are read into
    pinned slots, copied to HBM and decompressed there, one wave per frame
    (csrc/xtc_gpu.hip); up to ``n_slots`` batches decode concurrently ahead
    of the consumer (3 slots: one hardware queue each beside the consumer's,
    HIP's default being 4 per process).  ``decode="host"``: frames are decoded frame-parallel on
    ``n_threads`` host threads straight into the stager's pinned slots
    (selection applied) and DMA'd.  Both give the same float32 frames.

    ``cache=True`` (GPU decode): decoded frames stay resident in HBM, so a
    second sweep over the trajectory -- RMSF.py re-reads every frame for its
    second loop (RMSF.py:124) -- reads them from HBM instead of decoding
    again; ignored (with no error) when the trajectory would take more than
    half of the free device memory."""

    def __init__(self, path, sel=None, batch_frames: int | None = None, n_slots: int = 3, n_threads: int = 16,
                 decode: str = "gpu", cache: bool = False):
        from .xtc import XTCFile

        if decode not in ("gpu", "host"):
            raise ValueError("decode must be 'gpu' or 'host'")
        self.xtc = XTCFile(path)
        self.n_traj, self.n_atoms = self.xtc.n_frames, self.xtc.n_atoms
        sel_arr = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if sel_arr is not None and sel_arr.size and (sel_arr.min() < 0 or sel_arr.max() >= self.n_atoms):
            raise IndexError("selection index out of range")
        self.n_sel = self.n_atoms if sel_arr is None else len(sel_arr)
        self.decode_on = decode
        if decode == "gpu":
            if batch_frames is None:  # ~2 GB of decoded frames per slot
                batch_frames = max(1, min(4096, (2 << 30) // max(1, 12 * self.n_atoms)))
            self.decoder = XtcDecoder(self.xtc, batch_frames, n_slots, n_threads)
            self.cache = None
            self._gather = None  # scratch for scattered frame lists served from the cache
            if cache:
                need = 12 * self.n_atoms * self.n_traj
                free, _ = torch.cuda.mem_get_info()
                if need <= free // 2:
                    self.cache = torch.empty((self.n_traj, self.n_atoms, 3), dtype=torch.float32,
                                             device=torch.cuda.current_device())
                    self._cached = np.zeros(self.n_traj, dtype=bool)
            self.sel_dev = None
            if sel_arr is not None and not np.array_equal(sel_arr, np.arange(self.n_sel)):
                self.sel_dev = torch.as_tensor(sel_arr.astype(np.int32)).to(torch.cuda.current_device())
        else:
            if batch_frames is None:
                batch_frames = max(1, min(4096, (64 << 20) // max(1, 12 * self.n_sel)))
            self.stager = Stager(self.n_atoms, self.n_sel, sel_arr, batch_frames, n_slots, n_threads)
        self.batch_frames = batch_frames

    def holds(self, frame: int) -> bool:
        return 0 <= frame < self.n_traj

    def drop_cache(self) -> None:
        """Forget the HBM-resident frames (the next sweep decodes again)."""
        if self.decode_on == "gpu" and self.cache is not None:
            self._cached[:] = False

    def _stage(self, first: int, step: int, n: int, stream: int) -> Batch:
        if self.decode_on == "gpu" and self.cache is not None:
            fs = 3 * self.n_atoms
            ptr = self.cache.data_ptr() + 4 * fs * first
            rows = first + step * np.arange(n)
            release = None
            if not self._cached[rows].all():
                slot = self.decoder.decode_into(first, n, step, ptr, fs * step, stream)
                self._cached[rows] = True
                release = lambda: self.decoder.release(slot, stream)  # noqa: E731
            return Batch(ptr, fs * step, n, self.sel_dev, release)
        if self.decode_on == "gpu":
            slot, ptr = self.decoder.decode(first, n, step, stream)
            return Batch(ptr, 3 * self.n_atoms, n, self.sel_dev, lambda: self.decoder.release(slot, stream))
        slot, dptr = ctypes.c_int(), ctypes.c_void_p()
        call("rmsf_stager_stage_xtc", self.stager._h, self.xtc.handle, first, n, step, stream, ctypes.byref(slot),
             ctypes.byref(dptr))
        s = slot.value
        return Batch(dptr.value, 3 * self.n_sel, n, None, lambda: self.stager.release(s, stream))

    def _check(self) -> None:
        if self.decode_on == "gpu":
            try:
                self.decoder.synchronize()
            except Exception:
                if self.cache is not None:
                    self._cached[:] = False  # a corrupt frame left NaN rows: decode again next time
                raise

    def reference(self, frame: int, stream: int) -> Batch:
        if self.decode_on == "gpu" and self.cache is not None:
            # a reference frame costs one whole decode latency: decode the
            # frames after it in the same wait (one batch per slot), so the
            # sweep that follows finds them resident
            first = frame
            for _ in range(self.decoder.n_slots):
                if first >= self.n_traj:
                    break
                n = min(self.batch_frames, self.n_traj - first)
                self._stage(first, 1, n, stream).done()
                first += n
        b = self._stage(frame, 1, 1, stream)
        self._check()
        return b

    def _list_batch(self, part: np.ndarray, stream: int) -> Batch:
        """Frames ``part`` of an explicit frame list (scattered records):
        decoded as ONE batch (rmsf_xtcdec_decode_list) instead of one decode
        per run; with the HBM cache their rows are copied in."""
        fs = 3 * self.n_atoms
        slot, ptr = self.decoder.decode_list(part, stream)
        if self.cache is not None:
            w = 4 * fs
            k = 0
            for first, step, n in FrameList(self.n_traj, frames=part).runs(0, len(part), len(part)):
                call("rmsf_memcpy2d_d2d", self.cache.data_ptr() + w * first, w * step, ptr + w * k, w, w, n, stream)
                k += n
            self._cached[part] = True
        return Batch(ptr, fs, len(part), self.sel_dev, lambda: self.decoder.release(slot, stream))

    def _cached_list(self, part: np.ndarray, stream: int) -> Batch:
        """Frames ``part``, all resident in the HBM cache, gathered into one
        compact batch (a scratch buffer reused by the next gather: yield it
        before gathering again)."""
        if self._gather is None or self._gather.buf.shape[0] < len(part):
            self._gather = _Gather(self.n_sel, self.batch_frames, self.cache.device)
        return self._gather(self.cache.data_ptr(), 3 * self.n_atoms, part, self.sel_dev, stream)

    def batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        ahead = self.decoder.n_slots - 1 if self.decode_on == "gpu" else 0
        queue = []
        nb = min(max_frames, self.batch_frames)
        if self.decode_on == "gpu" and _scattered(frames, b0, b1, nb):
            idx = frames.idx[b0:b1]
            for i in range(0, len(idx), nb):
                part = idx[i:i + nb]
                if self.cache is not None and self._cached[part].all():
                    while queue:  # decodes in flight first; a gathered batch is never queued ahead
                        yield queue.pop(0)
                    yield self._cached_list(part, stream)
                    continue
                queue.append(self._list_batch(part, stream))
                while len(queue) > ahead:
                    yield queue.pop(0)
        else:
            for first, step, n in frames.runs(b0, b1, nb):
                queue.append(self._stage(first, step, n, stream))
                if len(queue) > ahead:
                    yield queue.pop(0)
        while queue:
            yield queue.pop(0)
        self._check()


class DcdSource:
    """CHARMM/NAMD/X-PLOR DCD file (BASELINE C1's adk trajectory format),
    streamed: each batch's selected rows are read from the memory-mapped file
    (the x/y/z planes interleaved on the host -- what RMSF.py:92,124's reader
    does per frame) and staged, so reading batch k+1 overlaps the copy and
    kernels of batch k and host memory stays bounded by the batch.  Native-
    endian files with every atom in every frame are staged straight from the
    map: the stager's threads gather the selection from the X/Y/Z records and
    interleave it into the pinned slot (rmsf_stager_stage_planes), with no
    intermediate array; other files are read by DCDFile.read first.
    ``cache=True``: FrameCache (RMSF.py's second loop reads HBM)."""

    def __init__(self, path, sel=None, batch_frames: int | None = None, n_slots: int = 3, cache: bool = False):
        from .dcd import DCDFile

        self.f = DCDFile(path)
        self.n_traj, self.n_atoms = len(self.f), self.f.n_atoms
        self.sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.sel is not None and self.sel.size and (self.sel.min() < 0 or self.sel.max() >= self.n_atoms):
            raise IndexError("selection index out of range")
        self.n_sel = self.n_atoms if self.sel is None else len(self.sel)
        if batch_frames is None:  # ~64 MB per slot
            batch_frames = max(1, min(4096, (64 << 20) // max(1, 12 * self.n_sel)))
        self.batch_frames = batch_frames
        self.planes = self.n_traj > 0 and self.f.plane_ptrs([0]) is not None
        if self.planes:  # the stager gathers the selection from the mapped planes
            self.stager = Stager(self.n_atoms, self.n_sel, self.sel, batch_frames, n_slots, 4)
        else:
            self.stager = Stager(self.n_sel, self.n_sel, None, batch_frames, n_slots, 1)
        ok = cache and FrameCache.fits(self.n_traj, self.n_sel)
        self.cache = FrameCache(self.n_traj, self.n_sel) if ok else None

    def holds(self, frame: int) -> bool:
        return 0 <= frame < self.n_traj

    def drop_cache(self) -> None:
        if self.cache is not None:
            self.cache.drop()

    def _stage_frames(self, frames: np.ndarray, stream: int) -> Batch:
        """Frames ``frames`` (any list) as one staged batch."""
        if self.planes:
            ptrs, plane_stride = self.f.plane_ptrs(frames)
            slot, ptr = self.stager.stage_planes(ptrs, plane_stride, stream)
        else:
            buf = np.concatenate([self.f.read(first, n, step, self.sel) for first, step, n in _list_runs(frames)])
            slot, ptr = self.stager.stage_compact(buf, len(frames), stream)  # copied into the pinned slot on return
        return Batch(ptr, 3 * self.n_sel, len(frames), None, lambda: self.stager.release(slot, stream))

    def _stage(self, first: int, step: int, n: int, stream: int) -> Batch:
        def stage():
            if self.planes:
                return self._stage_frames(first + step * np.arange(n, dtype=np.int64), stream)
            buf = np.ascontiguousarray(self.f.read(first, n, step, self.sel))
            slot, ptr = self.stager.stage_compact(buf, n, stream)  # copied into the pinned slot on return
            return Batch(ptr, 3 * self.n_sel, n, None, lambda: self.stager.release(slot, stream))

        return _cached_stage(self.cache, first, step, n, stream, stage)

    def reference(self, frame: int, stream: int) -> Batch:
        if not self.holds(frame):
            raise IndexError(f"frame {frame} out of range ({self.n_traj} frames)")
        return self._stage(frame, 1, 1, stream)

    def batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        nb = min(max_frames, self.batch_frames)
        if _scattered(frames, b0, b1, nb):
            g = _Gather(self.n_sel, nb, self.cache.buf.device) if self.cache is not None else None

            def stage(rows):
                return self._stage_frames(rows, stream)

            idx = frames.idx[b0:b1]
            for i in range(0, len(idx), nb):
                yield _cached_list(self.cache, g, idx[i:i + nb], stream, stage)
            return
        for first, step, n in frames.runs(b0, b1, nb):
            yield self._stage(first, step, n, stream)


class AtomGroupSource:
    """MDAnalysis AtomGroup: per-Timestep ``ag.positions`` (the selection rows,
    RMSF.py:95,128) packed into a host batch and staged to the device."""

    def __init__(self, atomgroup, batch_frames: int | None = None, n_slots: int = 3, cache: bool = False):
        self.ag = atomgroup
        self.traj = atomgroup.universe.trajectory
        self.n_traj = len(self.traj)
        self.n_sel = len(atomgroup)
        if batch_frames is None:
            batch_frames = max(1, min(1024, (32 << 20) // max(1, 12 * self.n_sel)))
        self.batch_frames = batch_frames
        self.stager = Stager(self.n_sel, self.n_sel, None, batch_frames, n_slots, 1)
        self._bufs = [np.empty((batch_frames, self.n_sel, 3), np.float32) for _ in range(n_slots)]
        self._next = 0
        # RMSF.py's second loop (RMSF.py:124) re-reads every Timestep: with a
        # cache the reader runs once per frame
        ok = cache and FrameCache.fits(self.n_traj, self.n_sel)
        self.cache = FrameCache(self.n_traj, self.n_sel) if ok else None

    def holds(self, frame: int) -> bool:
        return 0 <= frame < self.n_traj

    def drop_cache(self) -> None:
        if self.cache is not None:
            self.cache.drop()

    def _buf(self) -> np.ndarray:
        b = self._bufs[self._next]
        self._next = (self._next + 1) % len(self._bufs)
        return b

    def reference(self, frame: int, stream: int) -> Batch:
        def stage():
            cur = self.traj.ts.frame
            try:
                self.traj[frame]
                buf = self._buf()
                buf[0] = self.ag.positions
            finally:
                self.traj[cur]
            slot, ptr = self.stager.stage_compact(buf, 1, stream)
            return Batch(ptr, 3 * self.n_sel, 1, None, lambda: self.stager.release(slot, stream))

        return _cached_stage(self.cache, frame, 1, 1, stream, stage)

    def batches(self, frames: FrameList, b0: int, b1: int, max_frames: int, stream: int) -> Iterator[Batch]:
        nb = min(max_frames, self.batch_frames)
        if _scattered(frames, b0, b1, nb):
            g = _Gather(self.n_sel, nb, self.cache.buf.device) if self.cache is not None else None

            def stage_list(rows):
                buf = self._buf()
                for j, f in enumerate(rows):
                    self.traj[int(f)]
                    buf[j] = self.ag.positions
                slot, ptr = self.stager.stage_compact(buf, len(rows), stream)
                return Batch(ptr, 3 * self.n_sel, len(rows), None, lambda: self.stager.release(slot, stream))

            idx = frames.idx[b0:b1]
            for i in range(0, len(idx), nb):
                yield _cached_list(self.cache, g, idx[i:i + nb], stream, stage_list)
            return
        for first, step, n in frames.runs(b0, b1, nb):

            def stage(first=first, step=step, n=n):
                buf = self._buf()
                for j in range(n):
                    self.traj[first + j * step]
                    buf[j] = self.ag.positions
                slot, ptr = self.stager.stage_compact(buf, n, stream)
                return Batch(ptr, 3 * self.n_sel, n, None, lambda: self.stager.release(slot, stream))

            yield _cached_stage(self.cache, first, step, n, stream, stage)


__all__ = ["Batch", "Stager", "FrameCache", "FrameList", "DeviceSource", "HostSource", "DcdSource", "XtcDecoder", "XtcSource", "AtomGroupSource",
           "_lib"]
