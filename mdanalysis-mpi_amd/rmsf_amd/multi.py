"""One process, several GPUs: ``RMSF(..., gpus=N).run()`` without a launcher.

RMSF.py runs one MPI rank per frame block (RMSF.py:59-72) and merges with
``Allreduce`` (RMSF.py:110) and a pickle ``comm.reduce`` (RMSF.py:143).  Here
one Python process drives one context of the C ABI (``rmsf_ctx``, csrc/
context.cpp) per device, each owning the RMSF.py:65-69 block of its index;
the per-device work runs on one host thread per context (the ctypes calls
release the GIL), and the two exchange steps run over RCCL communicators made
by ``ncclCommInitAll`` (``rmsf_multi_init_all``) -- or, when a device appears
twice in ``gpus`` (one GPU hosting several blocks), over the contexts'
in-process fold, which performs the same arithmetic.

Per context, RMSF.py's rank loop in context-ABI terms:

    set_reference_frame(frame ref_frame)                 RMSF.py:80-87
    push(block, ALIGN_SUM)                               RMSF.py:89-105
    multi_allreduce_sum(all)                             RMSF.py:107-110
    set_reference_average()                              RMSF.py:111-118
    push(block, ALIGN_WELFORD)                           RMSF.py:120-138
    multi_chan_merge(all[, root])                        RMSF.py:140-143
    get_rmsf                                             RMSF.py:145-146

(``align=None``: one Welford push, with frame 0 of the frame list set on
every context as the merge's shift -- the one-collective merge, as the
torchrun pipeline's; ``"frame0"``: reference + aligned Welford.)
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import parallel
from .context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, PUSH_EXACT, PUSH_WELFORD, Context
from ._lib import RmsfEmptyError
from .sources import FrameList


def device_list(gpus) -> list[int]:
    """``gpus``: a count (devices 0..N-1) or an explicit list of device ids."""
    if isinstance(gpus, (int, np.integer)):
        if gpus < 1:
            raise ValueError("gpus must be >= 1")
        return list(range(int(gpus)))
    devs = [int(d) for d in gpus]
    if not devs or min(devs) < 0:
        raise ValueError("gpus: a non-empty list of device ids expected")
    return devs


class _HostFrames:
    """A float32 [F, n_atoms, 3] host trajectory (or [F, 3, n_atoms]
    coordinate planes, ``layout="soa"``); the contexts gather the selection
    (and interleave planes) into their stagers."""

    def __init__(self, arr: np.ndarray, sel, layout: str = "fac"):
        self.layout = layout
        if layout == "soa":
            if arr.dtype != np.float32 or arr.ndim != 3 or arr.shape[1] != 3:
                raise ValueError("SoA host trajectory must be float32 [n_frames, 3, n_atoms]")
            self.arr = np.ascontiguousarray(arr)
            self.n_traj, self.n_atoms = self.arr.shape[0], self.arr.shape[2]
        else:
            if arr.dtype != np.float32 or arr.ndim != 3 or arr.shape[2] != 3:
                raise ValueError("host trajectory must be float32 [n_frames, n_atoms, 3]")
            self.arr = np.ascontiguousarray(arr)
            self.n_traj, self.n_atoms = self.arr.shape[0], self.arr.shape[1]
        self.sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.sel is not None and self.sel.size and (self.sel.min() < 0 or self.sel.max() >= self.n_atoms):
            raise IndexError("selection index out of range")

    def reference(self, frame: int) -> np.ndarray:
        return np.ascontiguousarray(self.arr[frame].T) if self.layout == "soa" else self.arr[frame]

    def push(self, ctx: Context, rows: range, mode: int) -> None:
        if not len(rows):
            return
        if self.layout == "soa":
            ctx.push_planes(self.arr, np.arange(rows.start, rows.stop, rows.step), mode)
        else:
            # rows is an arithmetic range: a strided view, pushed with its step
            ctx.push(self.arr[rows.start:rows[-1] + 1], mode, step=rows.step)

    def push_block(self, ctx: Context, runs: list, mode: int) -> None:
        """A block of several runs (a scattered frame list): one push of one
        pointer per frame, batched by the stager, instead of one per run."""
        if len(runs) == 1:
            self.push(ctx, runs[0], mode)
        elif runs:
            rows = np.concatenate([np.arange(r.start, r.stop, r.step) for r in runs])
            if self.layout == "soa":
                ctx.push_planes(self.arr, rows, mode)
            else:
                ctx.push_rows(self.arr, rows, mode)

    def n_sel(self) -> int:
        return self.n_atoms if self.sel is None else len(self.sel)

    def stage_block(self, dev: int, runs: list):
        """The block's selected rows (``runs``: strided ranges of frames)
        staged once into HBM on ``dev`` (pinned stager, then a resident
        [n, n_sel, 3] tensor): RMSF.py's two loops (RMSF.py:92,124) then both
        read HBM (run_multi checks the fit first)."""
        import torch

        from .sources import FrameCache, Stager

        ns = self.n_sel()
        total = sum(len(r) for r in runs)
        if not total:
            return None
        with torch.cuda.device(dev):
            cache = FrameCache(total, ns, device=torch.device("cuda", dev))
            batch = max(1, min(4096, (64 << 20) // max(1, 12 * ns)))
            st = Stager(self.n_atoms, ns, self.sel, batch, 3, 4)
            stream = torch.cuda.current_stream(dev).cuda_stream
            try:
                # every frame of the block by address: a scattered frame list
                # fills whole stager batches too
                frames = np.concatenate([np.arange(r.start, r.stop, r.step) for r in runs])
                addr = (self.arr.ctypes.data + frames * self.arr.strides[0]).astype(np.uint64)
                for row in range(0, total, batch):
                    n = min(batch, total - row)
                    if self.layout == "soa":
                        slot, ptr = st.stage_planes(addr[row:row + n], self.arr.strides[1] // 4, stream)
                    else:
                        slot, ptr = st.stage_ptrs(addr[row:row + n], stream)
                    cache.fill(row, 1, n, ptr, stream)
                    st.release(slot, stream)
                torch.cuda.current_stream(dev).synchronize()
            finally:
                st.close()
        return cache.buf


class _XtcFrames:
    """A GROMACS XTC file: each context decompresses its block on its GPU."""

    def __init__(self, path: str, sel):
        from .xtc import XTCFile

        self.xtc = XTCFile(path)
        self.n_traj, self.n_atoms = self.xtc.n_frames, self.xtc.n_atoms
        self.sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.sel is not None and self.sel.size and (self.sel.min() < 0 or self.sel.max() >= self.n_atoms):
            raise IndexError("selection index out of range")

    def reference(self, frame: int) -> np.ndarray:
        return self.xtc.read(frame, 1)[0]

    def push(self, ctx: Context, rows: range, mode: int) -> None:
        if len(rows):
            ctx.push_xtc(self.xtc, rows.start, rows[-1] + 1, rows.step, mode)

    def push_block(self, ctx: Context, runs: list, mode: int) -> None:
        """A block of several runs: the scattered records are decoded in
        batches by one push (one wait), not one blocking decode per run."""
        if len(runs) == 1:
            self.push(ctx, runs[0], mode)
        elif runs:
            ctx.push_xtc_frames(self.xtc, np.concatenate([np.arange(r.start, r.stop, r.step) for r in runs]), mode)


class _DcdFrames:
    """A CHARMM/NAMD DCD file: each context reads only its block's runs from
    the memory-mapped file (``DCDFile.read`` of the selected rows), in
    batches, and pushes them through its stager -- host memory stays bounded
    by a batch, as for the single-device ``DcdSource``."""

    def __init__(self, path: str, sel, batch_frames: int | None):
        from .dcd import DCDFile

        self.f = DCDFile(path)
        self.n_traj, n_atoms = len(self.f), self.f.n_atoms
        self.rsel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.rsel is not None and self.rsel.size and (self.rsel.min() < 0 or self.rsel.max() >= n_atoms):
            raise IndexError("selection index out of range")
        # the reads apply the selection: contexts see selected rows only
        self.n_atoms = n_atoms if self.rsel is None else len(self.rsel)
        self.sel = None
        self.batch = batch_frames or max(1, min(4096, (64 << 20) // max(1, 12 * self.n_atoms)))

    def reference(self, frame: int) -> np.ndarray:
        return self.f.read(frame, 1, 1, self.rsel)[0]

    def n_sel(self) -> int:
        return self.n_atoms

    def push(self, ctx: Context, rows: range, mode: int) -> None:
        for i in range(0, len(rows), self.batch):
            part = rows[i:i + self.batch]
            ctx.push(self.f.read(part.start, len(part), part.step, self.rsel), mode)

    def stage_block(self, dev: int, runs: list):
        """The block's rows read batch by batch and staged into HBM once."""
        import torch

        from .sources import FrameCache, Stager

        total = sum(len(r) for r in runs)
        if not total:
            return None
        ns = self.n_atoms
        with torch.cuda.device(dev):
            cache = FrameCache(total, ns, device=torch.device("cuda", dev))
            st = Stager(ns, ns, None, self.batch, 3, 1)
            stream = torch.cuda.current_stream(dev).cuda_stream
            try:
                row = 0
                for rows in runs:
                    for i in range(0, len(rows), self.batch):
                        part = rows[i:i + self.batch]
                        buf = self.f.read(part.start, len(part), part.step, self.rsel)
                        slot, ptr = st.stage_compact(buf, len(part), stream)
                        cache.fill(row, 1, len(part), ptr, stream)
                        st.release(slot, stream)
                        row += len(part)
                torch.cuda.current_stream(dev).synchronize()
            finally:
                st.close()
        return cache.buf


class _DeviceShards:
    """An HBM-resident trajectory held as one float32 [F_i, n_atoms, 3] torch
    tensor per device; concatenated in the given order they are the
    trajectory.  Each device's context processes the frames of the frame
    list that lie in its own shard ("owner computes": no frame crosses
    xGMI), and the exchanges merge them as they merge RMSF.py's blocks."""

    def __init__(self, tensors, sel):
        import torch

        self.parts = list(tensors)
        if not self.parts:
            raise ValueError("no device shards")
        for t in self.parts:
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.dim() == 3
                    and t.shape[2] == 3 and t.is_contiguous()):
                raise TypeError("device shards must be contiguous float32 HIP tensors [n_frames, n_atoms, 3]")
        self.n_atoms = self.parts[0].shape[1]
        if any(t.shape[1] != self.n_atoms for t in self.parts):
            raise ValueError("device shards differ in their atom count")
        self.devices = [t.device.index for t in self.parts]
        self.offsets = np.concatenate([[0], np.cumsum([t.shape[0] for t in self.parts])]).astype(np.int64)
        self.n_traj = int(self.offsets[-1])
        self.sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        if self.sel is not None and self.sel.size and (self.sel.min() < 0 or self.sel.max() >= self.n_atoms):
            raise IndexError("selection index out of range")

    def reference(self, frame: int):
        i = int(np.searchsorted(self.offsets, frame, side="right") - 1)
        return self.parts[i][frame - int(self.offsets[i])]

    def owner_blocks(self, fl: FrameList) -> list[tuple[int, int]]:
        """Positions [p0, p1) of the frame list inside each shard."""
        pos = np.array([fl[i] for i in range(len(fl))], dtype=np.int64) if fl.r is None else None
        out = []
        for i in range(len(self.parts)):
            lo, hi = int(self.offsets[i]), int(self.offsets[i + 1])
            if pos is None:
                r = fl.r
                p0 = len(range(r.start, lo, r.step)) if lo > r.start else 0
                p1 = len(range(r.start, hi, r.step)) if hi > r.start else 0
                out.append((min(p0, len(r)), min(p1, len(r))))
            else:
                out.append((int(np.searchsorted(pos, lo)), int(np.searchsorted(pos, hi))))
        return out

    def push_on(self, i: int, ctx: Context, rows: range, mode: int) -> None:
        if len(rows):
            off = int(self.offsets[i])
            ctx.push(self.parts[i][rows.start - off:rows[-1] - off + 1], mode, step=rows.step)


class _AtomGroupFrames:
    """An MDAnalysis AtomGroup: ``ag.positions`` per Timestep (RMSF.py:95,128),
    gathered on this thread (readers are not thread-safe) in batches."""

    serial = True

    def __init__(self, ag, batch_frames: int | None):
        self.ag, self.traj = ag, ag.universe.trajectory
        self.n_traj, self.n_atoms, self.sel = len(self.traj), len(ag), None
        self.batch = batch_frames or max(1, min(1024, (32 << 20) // max(1, 12 * self.n_atoms)))

    def reference(self, frame: int) -> np.ndarray:
        cur = self.traj.ts.frame
        try:
            self.traj[frame]
            return np.array(self.ag.positions, dtype=np.float32)
        finally:
            self.traj[cur]

    def push(self, ctx: Context, rows: range, mode: int) -> None:
        buf = np.empty((min(self.batch, max(1, len(rows))), self.n_atoms, 3), np.float32)
        for i in range(0, len(rows), self.batch):
            part = rows[i:i + self.batch]
            for j, f in enumerate(part):
                self.traj[f]
                buf[j] = self.ag.positions
            ctx.push(buf[:len(part)], mode)


def _blocks_fit(devs, blocks, n_sel: int) -> bool:
    """Every device can hold its blocks' selected rows in half its free HBM."""
    import torch

    need = {}
    for d, runs in zip(devs, blocks):
        need[d] = need.get(d, 0) + 12 * sum(len(r) for r in runs) * n_sel
    return all(n <= torch.cuda.mem_get_info(d)[0] // 2 for d, n in need.items())


def _frames_of(inp, sel, batch_frames, layout: str = "fac"):
    import os

    if isinstance(inp, np.ndarray):
        return _HostFrames(inp, sel, layout)
    if isinstance(inp, (list, tuple)) or (hasattr(inp, "is_cuda") and inp.is_cuda):
        return _DeviceShards([inp] if hasattr(inp, "is_cuda") else inp, sel)
    if isinstance(inp, (str, bytes)) or hasattr(inp, "__fspath__"):
        path = os.fspath(inp)
        if str(path).lower().endswith(".xtc"):
            return _XtcFrames(path, sel)
        if str(path).lower().endswith(".dcd"):
            return _DcdFrames(path, sel, batch_frames)
        raise ValueError(f"only .xtc and .dcd trajectory files are read natively, got {path!r}")
    if hasattr(inp, "universe") and hasattr(inp, "positions"):
        return _AtomGroupFrames(inp, batch_frames)
    raise TypeError(f"gpus=: unsupported input {type(inp)!r} (numpy array, .xtc/.dcd path, AtomGroup, or HIP "
                    "tensors -- one shard per device)")


def _set_frame(c: Context, fr, setter: str) -> None:
    """``setter`` (set_reference_frame / set_merge_shift_frame) of a frame
    that may live on another device: copied over xGMI on torch's stream of
    c's device; the setter orders the context stream after the copy and keeps
    the copy alive until the context is synchronised."""
    if hasattr(fr, "is_cuda") and fr.device.index != c.device:
        import torch
        with torch.cuda.device(c.device):
            getattr(c, setter)(fr.to(torch.device("cuda", c.device)))
    else:
        getattr(c, setter)(fr)


def _exact_merge(ctxs, root: int, order: str) -> dict:
    """RMSF.py:141-146 for exact=True: the contexts' states (each a block's S
    of RMSF.py:140) reduced with second_order_moments (RMSF.py:36-41 bit for
    bit) in RMSF.py:143's comm.reduce order, device to device
    (rmsf_multi_chan_merge_exact: each step's state crosses xGMI by a peer
    copy and merges on the receiving device), to context ``root``; then
    RMSF.py:146 there."""
    Context.multi_chan_merge_exact(ctxs, root=root, order=order)
    home = ctxs[root]
    n, mean, m2 = home.partial()
    return dict(rmsf=home.rmsf(), mean=mean, sumsquares=m2, n_frames=n)


def run_multi(inp, gpus, *, select=None, align=None, masses=None, ref_frame: int = 0, start=None, stop=None,
              step=None, batch_frames: int | None = None, frames=None, collect_rmsd: bool = False,
              layout: str = "fac", merge_root: int | None = None, exact: bool | None = None,
              merge_order: str = "mpi4py") -> dict:
    """RMSF.py's computation over the devices ``gpus`` from one process.
    Returns the ``results`` fields (rmsf, mean, sumsquares, n_frames, ...;
    ``rmsd`` with ``collect_rmsd``: per-frame QCP rmsd of the last sweep in
    frame-list order, the by-product RMSF.py:48 discards).  ``merge_root``:
    the final merge is a reduce to that device index (RMSF.py:143's shape)
    and the results are read from it; None = an all-reduce, read from
    device index 0 (the same numbers).  ``exact``: every device runs
    RMSF.py's statements over its block in the reference's summation orders
    (rmsf_ctx_set_exact: the sequential references, superposition and
    accumulate; align=None: RMSF.py:137-138's recurrence, RMSF_PUSH_EXACT),
    the sweep-1 sums meet in rank order, and the blocks are reduced by
    second_order_moments in ``merge_order`` (RMSF.py:143's comm.reduce:
    "mpi4py", its default binomial tree -- restated from mpi4py's published
    source, unverified here -- or "rank"), device to device: the script's
    arithmetic bit for bit."""
    from ._lib import merge_order as _order
    _order(merge_order)
    if align not in (None, "frame0", "average"):
        raise ValueError(f"align must be one of (None, 'frame0', 'average'), got {align!r}")
    if parallel.world()[1] > 1:
        raise ValueError("gpus= drives several devices from one process; under torch.distributed "
                         "(one process per GPU) leave it unset")
    if collect_rmsd and align is None:
        raise ValueError("collect_rmsd needs an aligned run (align='frame0' or 'average')")
    if layout == "soa" and not isinstance(inp, np.ndarray):
        raise NotImplementedError("gpus=: SoA input is supported for host numpy arrays [F, 3, n_atoms]")
    src = _frames_of(inp, select, batch_frames, layout)
    n_dev = len(src.parts) if isinstance(src, _DeviceShards) else len(device_list(gpus))
    if merge_root is not None and not 0 <= merge_root < n_dev:
        raise ValueError(f"merge_root {merge_root} is not one of the {n_dev} devices")
    fl = FrameList(src.n_traj, start, stop, step, frames=frames)
    if len(fl) == 0:
        raise RmsfEmptyError(-4, "RMSF.run", "no frames selected")
    if exact is None:  # the pipeline's default: exact for few-frame aligned runs
        from .pipeline import auto_exact
        exact = auto_exact(align, len(fl))
    if align is not None and not 0 <= ref_frame < src.n_traj:
        raise IndexError(f"ref_frame {ref_frame} outside the trajectory ({src.n_traj} frames)")
    if masses is None and align is not None and isinstance(src, _AtomGroupFrames):
        masses = np.asarray(src.ag.masses, dtype=np.float64)
    big = max(1, len(fl))
    if isinstance(src, _DeviceShards):
        # the data decide the placement: device i takes the frames in its shard
        devs = src.devices
        if gpus is not None and not isinstance(gpus, (int, np.integer)) and device_list(gpus) != devs:
            raise ValueError(f"gpus={list(gpus)} does not match the shards' devices {devs}")
        if isinstance(gpus, (int, np.integer)) and int(gpus) != len(devs):
            raise ValueError(f"gpus={gpus} but {len(devs)} device shards were given")
        spans = src.owner_blocks(fl)
    else:
        devs = device_list(gpus)
        spans = parallel.blocks(len(fl), len(devs))   # RMSF.py:65-69 over the frame list
    # each device's block of the frame list, as strided runs
    blocks = [[range(f, f + s * n, s) for f, s, n in fl.runs(b0, b1, big)] for b0, b1 in spans]
    # RMSF.py's two sweeps over host frames: each device stages its block's
    # selected rows into HBM once and both sweeps read them there (contexts
    # over the selection only: the in-kernel gather becomes the identity)
    staged = (align == "average" and isinstance(src, (_HostFrames, _DcdFrames))
              and _blocks_fit(devs, blocks, src.n_sel()))
    if staged:
        ctxs = [Context(src.n_sel(), sel=None, masses=masses, device=d) for d in devs]
    else:
        ctxs = [Context(src.n_atoms, sel=src.sel, masses=masses, device=d) for d in devs]
    try:
        if exact and align is not None:
            for c in ctxs:
                c.set_exact(True, masses)
        if len(set(devs)) == len(devs) and len(devs) > 1:
            Context.init_all(ctxs)  # ncclCommInitAll: one communicator per device
        if collect_rmsd:
            for c in ctxs:
                c.collect_rmsd(True)

        def each(fn):
            if getattr(src, "serial", False) or len(ctxs) == 1:
                for i in range(len(ctxs)):
                    fn(i)
                return
            with ThreadPoolExecutor(len(ctxs)) as ex:
                for f in [ex.submit(fn, i) for i in range(len(ctxs))]:
                    f.result()

        out = {}
        if align is not None:
            ref = src.reference(ref_frame)
            if staged and getattr(src, "sel", None) is not None:
                ref = ref[src.sel]
            for c in ctxs:  # every rank reads the reference frame (RMSF.py:80-87)
                _set_frame(c, ref, "set_reference_frame")
        elif len(ctxs) > 1 and not exact:
            # the merge's shift: frame 0 of the frame list on every context
            # (the one-collective merge, as the torchrun pipeline's)
            shift = src.reference(fl[0])
            for c in ctxs:
                _set_frame(c, shift, "set_merge_shift_frame")
        cached = {}
        if staged:
            def stage(i):
                cached[i] = src.stage_block(ctxs[i].device, blocks[i])
            each(stage)

        def push(i, mode):
            c = ctxs[i]
            if staged:
                if cached[i] is not None:
                    c.push(cached[i], mode)
            elif isinstance(src, _DeviceShards):
                for r in blocks[i]:
                    src.push_on(i, c, r, mode)
            elif hasattr(src, "push_block"):
                src.push_block(c, blocks[i], mode)
            else:
                for r in blocks[i]:
                    src.push(c, r, mode)

        # HBM shards whose device blocks are single unit-step runs: one
        # rmsf_multi_push_frames call (every context's launches from its own
        # host thread; from 1M atoms the unaligned sweep runs in atom slabs
        # beside the merge's collectives)
        whole = (isinstance(src, _DeviceShards) and not staged and not exact
                 and all(len(runs) <= 1 and all(r.step == 1 for r in runs) for runs in blocks))

        def multi_push(mode):
            parts = []
            for i, runs in enumerate(blocks):
                t = src.parts[i]
                if runs:
                    off = int(src.offsets[i])
                    parts.append(t[runs[0].start - off:runs[0].stop - off])
                else:
                    parts.append(t[:0])
            Context.multi_push_frames(ctxs, parts, mode, reset=False)

        if align == "average":
            if whole:
                multi_push(PUSH_ALIGN_SUM)
            else:
                each(lambda i: push(i, PUSH_ALIGN_SUM))
            Context.multi_allreduce_sum(ctxs)
            for c in ctxs:
                c.set_reference_average()
            out["average"] = ctxs[0].average().reshape(-1)  # flat, as the pipeline returns it
        if collect_rmsd:
            for c in ctxs:  # the last sweep's rmsd only, as the pipeline reports it
                c.collect_rmsd(True)
        last = PUSH_WELFORD if align is None else PUSH_ALIGN_WELFORD
        if exact and align is None:
            last = PUSH_EXACT
        if whole:
            multi_push(last)
        else:
            each(lambda i: push(i, last))
        if exact:
            out.update(_exact_merge(ctxs, merge_root or 0, merge_order),
                       blocks=[(int(b0), int(b1)) for b0, b1 in spans], devices=devs, merge_order=merge_order)
            if collect_rmsd:
                out["rmsd"] = np.concatenate([c.rmsd() for c in ctxs])
            return out
        Context.multi_chan_merge(ctxs, root=merge_root)
        home = ctxs[merge_root or 0]
        n, mean, m2 = home.partial()
        out.update(rmsf=home.rmsf(), mean=mean, sumsquares=m2, n_frames=n,
                   blocks=[(int(b0), int(b1)) for b0, b1 in spans], devices=devs)
        if collect_rmsd:
            out["rmsd"] = np.concatenate([c.rmsd() for c in ctxs])
        return out
    finally:
        for c in ctxs:
            c.close()
