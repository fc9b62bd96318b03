"""``Context`` -- the C ABI's RMSF context (rmsf_ctx_*) from Python.

The context API is the torch-free boundary of include/rmsf_hip.h: one opaque
handle per device owning the selection, reference, running Welford / sweep-1
sum partials, a pinned stager and a stream.  RMSF.py's per-rank loop
(RMSF.py:80-146) in these terms::

    c = Context(n_atoms, sel=ca.indices, masses=None, device=0)
    c.set_reference_frame(frame0)                      # RMSF.py:80-87
    c.push(block, PUSH_ALIGN_SUM)                      # RMSF.py:89-105
    c.allreduce_sum()                                  # RMSF.py:107-110
    c.set_reference_average()                          # RMSF.py:111-118
    c.push(block, PUSH_ALIGN_WELFORD)                  # RMSF.py:120-138
    c.chan_merge()                                     # RMSF.py:140-143
    rmsf = c.rmsf()                                    # RMSF.py:145-146

Frames are numpy float32 [n, n_atoms, 3] (host: gathered and streamed by the
stager) or HIP torch tensors (device: read in place).  Exchanges run over a
torch.distributed process group when one is initialised with world > 1
(through the C callback transport), otherwise over the contexts of this
process (``Context.multi_*``: RCCL when ``init_rccl``/``init_all`` gave them
communicators, else an in-process host fold).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import (ALLREDUCE_FN, RMSF_MULTI_RESET, RMSF_PUSH_ALIGN_SUM, RMSF_PUSH_ALIGN_WELFORD, RMSF_PUSH_EXACT,
                   RMSF_PUSH_SUM, RMSF_PUSH_WELFORD, RMSF_TIME_ACCUMULATE, RMSF_TIME_MERGE, RMSF_TIME_SUPERPOSE,
                   RMSF_TRANSPORT_AUTO, RMSF_TRANSPORT_NOOP, RMSF_UNIQUE_ID_BYTES, call, load)

PUSH_WELFORD = RMSF_PUSH_WELFORD
PUSH_ALIGN_SUM = RMSF_PUSH_ALIGN_SUM
PUSH_ALIGN_WELFORD = RMSF_PUSH_ALIGN_WELFORD
PUSH_SUM = RMSF_PUSH_SUM
PUSH_EXACT = RMSF_PUSH_EXACT  # RMSF.py:137-138 as written (rmsf_welford_sequential)
TRANSPORT_AUTO = RMSF_TRANSPORT_AUTO
TRANSPORT_NOOP = RMSF_TRANSPORT_NOOP


def _f64(a, n: int, name: str) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.size != n:
        raise ValueError(f"{name}: expected {n} values, got {a.size}")
    return a


def dist_allreduce(d_buf: int, count: int, stream: int, user) -> int:
    """rmsf_allreduce_fn over the default torch.distributed group: the
    device buffer is staged through host memory (a once-per-run exchange of
    3*n_sel doubles) and summed with dist.all_reduce."""
    import torch
    import torch.distributed as dist

    try:
        host = np.empty(count, dtype=np.float64)
        call("rmsf_memcpy_d2h", host.ctypes.data, d_buf, 8 * count, stream)
        call("rmsf_stream_synchronize", stream)
        t = torch.from_numpy(host)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t)
        host[:] = t.cpu().numpy()
        call("rmsf_memcpy_h2d", d_buf, host.ctypes.data, 8 * count, stream)
        call("rmsf_stream_synchronize", stream)
        return 0
    except Exception:  # noqa: BLE001 -- no exception may cross the C callback
        return 1


_DIST_FN = ALLREDUCE_FN(lambda b, n, s, u: dist_allreduce(b, n, s, u))


def _dist_world() -> int:
    try:
        import torch.distributed as dist
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    except Exception:  # noqa: BLE001
        return 1


class Context:
    def __init__(self, n_atoms: int, sel=None, masses=None, device: int = 0, n_sel: int | None = None):
        load()
        self.n_atoms = int(n_atoms)
        self._sel = None if sel is None else np.ascontiguousarray(sel, dtype=np.int64)
        self.n_sel = len(self._sel) if self._sel is not None else int(n_sel if n_sel is not None else n_atoms)
        m = None if masses is None else _f64(masses, self.n_sel, "masses")
        self.device = device
        self._alive = {}     # device tensors read by queued work, by id (released at the next synchronisation)
        self._ext = None     # torch's view of the context stream (cached)
        self._h = ctypes.c_void_p()
        call("rmsf_ctx_create", device, self.n_atoms, self.n_sel,
             None if self._sel is None else self._sel.ctypes.data, None if m is None else m.ctypes.data, 0,
             ctypes.byref(self._h))

    # -- lifecycle ------------------------------------------------------------
    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    @property
    def stream(self) -> int:
        s = ctypes.c_void_p()
        call("rmsf_ctx_stream", self._h, ctypes.byref(s))
        return s.value or 0

    def close(self) -> None:
        if self._h:
            call("rmsf_ctx_destroy", self._h)  # synchronises the context stream first
            self._h = ctypes.c_void_p()
        self._alive.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def synchronize(self) -> None:
        call("rmsf_ctx_synchronize", self._h)
        self._alive.clear()

    def set_staging(self, batch_frames: int = 0, n_slots: int = 2, n_threads: int = 4) -> None:
        call("rmsf_ctx_set_staging", self._h, batch_frames, n_slots, n_threads)

    def set_timing(self, on: bool = True) -> None:
        """HIP events around every superpose / accumulate launch and around
        this context's part of each cross-context merge (measurement)."""
        call("rmsf_ctx_set_timing", self._h, 1 if on else 0)

    def kernel_time(self, which: str = "accumulate") -> tuple[int, float, float]:
        """(launches, summed ms, atom-frames) of one kernel family since the
        last call (``which``: "accumulate", "superpose", or "merge" -- the
        context's merges: from its packed moments to its finished result,
        atom-frames 0); synchronises."""
        k = {"accumulate": RMSF_TIME_ACCUMULATE, "superpose": RMSF_TIME_SUPERPOSE, "merge": RMSF_TIME_MERGE}[which]
        n, ms, af = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
        call("rmsf_ctx_kernel_time", self._h, k, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(af))
        self._alive.clear()  # kernel_time synchronised the stream
        return n.value, ms.value, af.value

    def collect_rmsd(self, on: bool = True) -> None:
        """Keep the per-frame QCP rmsd of aligned Welford pushes (RMSF.py:48)."""
        call("rmsf_ctx_collect_rmsd", self._h, 1 if on else 0)

    def rmsd(self) -> np.ndarray:
        n = ctypes.c_int64()
        call("rmsf_get_rmsd", self._h, ctypes.byref(n), None, 0)
        out = np.empty(n.value)
        if n.value:
            call("rmsf_get_rmsd", self._h, ctypes.byref(n), out.ctypes.data, out.size)
        return out

    def set_exact(self, on: bool = True, masses=None) -> None:
        """exact=True (rmsf_ctx_set_exact): references, aligned pushes and
        the sweep-1 sum exchange in RMSF.py's own summation orders.  The
        centre of mass divides by numpy's ``masses.sum()`` of the selection
        (``masses``: the context's, default unit masses -> n_sel).  Call it
        before setting the reference."""
        mt = float(np.ascontiguousarray(masses, dtype=np.float64).sum()) if masses is not None else float(self.n_sel)
        call("rmsf_ctx_set_exact", self._h, 1 if on else 0, mt)

    def reset(self, welford: bool = True, sum: bool = True) -> None:  # noqa: A002
        call("rmsf_ctx_reset", self._h, (1 if welford else 0) | (2 if sum else 0))

    # -- reference ------------------------------------------------------------
    def set_reference(self, ref_centered, ref_com) -> None:
        r = _f64(ref_centered, 3 * self.n_sel, "ref_centered")
        c = _f64(ref_com, 3, "ref_com")
        call("rmsf_set_reference", self._h, r.ctypes.data, c.ctypes.data)

    def set_reference_frame(self, frame) -> None:
        ptr, dev, keep = self._frames_ptr(frame, 1)
        call("rmsf_set_reference_frame", self._h, ptr, dev)
        if dev:
            # the setup kernels read the frame asynchronously on the context
            # stream: a temporary (e.g. a copy from another device) must
            # outlive them
            self._alive[id(keep)] = keep

    def set_merge_shift_frame(self, frame) -> None:
        """The merge's shift for unaligned Welford state: frame 0 of the frame
        list (all n_atoms atoms; the context keeps its selected rows), the
        same on every context (rmsf_set_merge_shift_frame)."""
        ptr, dev, keep = self._frames_ptr(frame, 1)
        call("rmsf_set_merge_shift_frame", self._h, ptr, dev)
        if dev:
            self._alive[id(keep)] = keep

    def set_reference_average(self) -> None:
        call("rmsf_set_reference_average", self._h)

    # -- frames ---------------------------------------------------------------
    def _frames_ptr(self, frames, expect_frames: int | None = None):
        """(pointer, is_device, keep-alive) for numpy host or HIP torch frames."""
        if hasattr(frames, "is_cuda") and frames.is_cuda:
            import torch
            if frames.dtype != torch.float32 or not frames.is_contiguous():
                raise ValueError("device frames must be contiguous float32")
            if frames.numel() % (3 * self.n_atoms):
                raise ValueError(f"device frames: not a whole number of {self.n_atoms}-atom frames")
            self._after_torch(frames)
            return frames.data_ptr(), 1, frames
        a = np.ascontiguousarray(frames, dtype=np.float32)
        if a.size % (3 * self.n_atoms):
            raise ValueError(f"host frames: not a whole number of {self.n_atoms}-atom frames")
        return a.ctypes.data, 0, a

    def _after_torch(self, t) -> None:
        """Order the context stream after the work torch has queued on the
        tensor's device (a copy or kernel that produces ``t``): the context
        reads device frames on its own non-blocking stream, which nothing else
        orders behind torch's current stream.  An event wait, no host sync."""
        import torch

        if self._ext is None:
            with torch.cuda.device(self.device):
                self._ext = torch.cuda.ExternalStream(self.stream, device=torch.device("cuda", self.device))
        self._ext.wait_stream(torch.cuda.current_stream(t.device))

    def push(self, frames, mode: int = PUSH_WELFORD, step: int = 1) -> None:
        """Push frames [n, n_atoms, 3] (every ``step``-th one)."""
        ptr, dev, keep = self._frames_ptr(frames)
        n_all = keep.numel() if dev else keep.size
        n_all //= 3 * self.n_atoms
        n = len(range(0, n_all, step))
        call("rmsf_push_frames", self._h, ptr, n, 3 * self.n_atoms * step, mode, dev)
        if dev:
            # device frames are read asynchronously: the tensor is kept alive
            # until the context is next synchronised (no host sync here)
            self._alive[id(keep)] = keep

    def push_xtc(self, xtc, start: int = 0, stop: int | None = None, step: int = 1, mode: int = PUSH_WELFORD):
        stop = xtc.n_frames if stop is None else min(stop, xtc.n_frames)
        n = len(range(start, stop, step))
        call("rmsf_push_xtc", self._h, xtc.handle, start, n, step, mode)

    def push_xtc_frames(self, xtc, frames, mode: int = PUSH_WELFORD) -> None:
        """Push the XTC frames ``frames`` (a frame list: scattered records are
        read and decoded in batches, one wait at the end)."""
        f = np.ascontiguousarray(frames, dtype=np.int64)
        call("rmsf_push_xtc_frames", self._h, xtc.handle, f.ctypes.data, f.size, mode)

    def push_rows(self, frames: np.ndarray, rows, mode: int = PUSH_WELFORD) -> None:
        """Push rows ``rows`` of a host float32 trajectory [F, n_atoms, 3]
        (any frame list) as one pointer per frame through the stager."""
        a = frames
        if a.dtype != np.float32 or not a.flags.c_contiguous or a.ndim != 3 or a.shape[1] != self.n_atoms:
            raise ValueError("push_rows: a C-contiguous float32 [F, n_atoms, 3] host array is required")
        r = np.asarray(rows, dtype=np.int64)
        if r.size and (r.min() < 0 or r.max() >= a.shape[0]):
            raise IndexError("push_rows: row out of range")
        ptrs = (a.ctypes.data + r * (a.strides[0])).astype(np.uint64)
        call("rmsf_push_frame_ptrs", self._h, ptrs.ctypes.data, r.size, mode)

    def push_planes(self, frames: np.ndarray, rows, mode: int = PUSH_WELFORD) -> None:
        """Push rows ``rows`` of a host float32 trajectory stored as
        coordinate planes, [F, 3, n_atoms] (SoA: x, y, z planes per frame),
        through the stager, which interleaves the selection on the host."""
        a = frames
        if a.dtype != np.float32 or a.ndim != 3 or a.shape[1] != 3 or a.shape[2] != self.n_atoms:
            raise ValueError("push_planes: a float32 [F, 3, n_atoms] host array is required")
        s0, s1, s2 = a.strides
        # the stager reads plane p of frame f at ptr[f] + p * plane_stride
        # floats, n_atoms contiguous floats each: any other view is copied
        if s2 != 4 or s1 < 0 or s0 < 0 or s1 % 4 or s0 % 4 or s1 < 4 * self.n_atoms or s0 < 3 * s1:
            a = np.ascontiguousarray(a)
        r = np.asarray(rows, dtype=np.int64)
        if r.size and (r.min() < 0 or r.max() >= a.shape[0]):
            raise IndexError("push_planes: row out of range")
        ptrs = (a.ctypes.data + r * a.strides[0]).astype(np.uint64)
        call("rmsf_push_frame_planes", self._h, ptrs.ctypes.data, a.strides[1] // 4, r.size, mode)

    # -- results --------------------------------------------------------------
    def partial(self):
        n = ctypes.c_int64()
        mean = np.empty((self.n_sel, 3))
        m2 = np.empty((self.n_sel, 3))
        call("rmsf_get_partial", self._h, ctypes.byref(n), mean.ctypes.data, m2.ctypes.data)
        self._alive.clear()  # the getters synchronise the context stream
        return n.value, mean, m2

    def sum(self):
        n = ctypes.c_int64()
        s = np.empty((self.n_sel, 3))
        call("rmsf_get_sum", self._h, ctypes.byref(n), s.ctypes.data)
        self._alive.clear()  # the getters synchronise the context stream
        return n.value, s

    def average(self) -> np.ndarray:
        out = np.empty((self.n_sel, 3))
        call("rmsf_get_average", self._h, out.ctypes.data)
        self._alive.clear()  # the getters synchronise the context stream
        return out

    def rmsf(self) -> np.ndarray:
        out = np.empty(self.n_sel)
        call("rmsf_get_rmsf", self._h, out.ctypes.data)
        self._alive.clear()  # the getters synchronise the context stream
        return out

    def set_partial(self, n: int, mean, m2) -> None:
        a = _f64(mean, 3 * self.n_sel, "mean")
        b = _f64(m2, 3 * self.n_sel, "m2")
        call("rmsf_set_partial", self._h, n, a.ctypes.data, b.ctypes.data)

    # -- exchange -------------------------------------------------------------
    def allreduce_sum(self, fn=None) -> None:
        """Sweep-1 sum + count over ranks (RMSF.py:107-110).  ``fn``: a ctypes
        ALLREDUCE_FN; default: torch.distributed when world > 1, else a no-op
        fold of this one context."""
        if fn is None and _dist_world() > 1:
            fn = _DIST_FN
        if fn is None:
            Context.multi_allreduce_sum([self])
        else:
            call("rmsf_ctx_allreduce_sum", self._h, ctypes.cast(fn, ctypes.c_void_p), None)

    def chan_merge(self, fn=None, shifted: bool = False) -> None:
        """Exact k-way Chan merge over ranks (RMSF.py:140-143).  ``shifted``:
        one data all-reduce of moments about the reference every rank holds
        (rmsf_ctx_chan_merge_shifted; all ranks must pass the same choice)
        instead of two."""
        if fn is None and _dist_world() > 1:
            fn = _DIST_FN
        if fn is None:
            Context.multi_chan_merge([self])
        else:
            name = "rmsf_ctx_chan_merge_shifted" if shifted else "rmsf_ctx_chan_merge"
            call(name, self._h, ctypes.cast(fn, ctypes.c_void_p), None)

    # -- RCCL / in-process groups ---------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(RMSF_UNIQUE_ID_BYTES)
        call("rmsf_multi_unique_id", buf)
        return buf.raw

    def init_rccl(self, uid: bytes, nranks: int, rank: int) -> None:
        if len(uid) != RMSF_UNIQUE_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        buf = ctypes.create_string_buffer(uid, RMSF_UNIQUE_ID_BYTES)
        call("rmsf_multi_init", self._h, buf, nranks, rank)

    @staticmethod
    def _handles(ctxs):
        arr = (ctypes.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
        return arr, len(ctxs)

    @staticmethod
    def init_all(ctxs) -> None:
        call("rmsf_multi_init_all", *Context._handles(ctxs))

    @staticmethod
    def multi_allreduce_sum(ctxs) -> None:
        call("rmsf_multi_allreduce_sum", *Context._handles(ctxs))

    @staticmethod
    def multi_chan_merge(ctxs, root: int | None = None) -> None:
        """RMSF.py:140-143 over the contexts: root=None leaves the result in
        every context (rmsf_multi_chan_merge); root=r reduces it to context
        r only, as RMSF.py:143's comm.reduce(root=0) (the others then refuse
        rmsf() until reset)."""
        h, n = Context._handles(ctxs)
        call("rmsf_multi_chan_merge_root", h, n, -1 if root is None else int(root))

    @staticmethod
    def multi_chan_merge_exact(ctxs, root: int | None = None, order="mpi4py") -> None:
        """RMSF.py:141-143 as the script computes it, over contexts holding
        ranks' exact states (PUSH_EXACT; context i = rank i): the states are
        reduced with second_order_moments in ``order`` ("mpi4py": comm.reduce's
        default binomial tree; "rank": rank order), device to device (peer
        copies, rmsf_multi_chan_merge_exact) -- bit for bit with RMSF.py:143.
        root=None: every context gets the result; root=r: context r only."""
        from ._lib import merge_order
        h, n = Context._handles(ctxs)
        call("rmsf_multi_chan_merge_exact", h, n, -1 if root is None else int(root), merge_order(order))

    @staticmethod
    def multi_set_transport(ctxs, transport: int) -> None:
        """TRANSPORT_AUTO (RCCL / host fold) or TRANSPORT_NOOP (timing
        rehearsal: the exchanges move nothing, results are not global)."""
        call("rmsf_multi_set_transport", *Context._handles(ctxs), int(transport))

    @staticmethod
    def multi_push_frames(ctxs, frames, mode: int = PUSH_WELFORD, *, reset: bool = True, ref_frames=None,
                          shift_frames=None, merge_slabs: int = 0, after_torch: bool = True) -> None:
        """Push HIP tensor ``frames[i]`` ([n_i, n_atoms, 3] float32,
        contiguous) to context i, every context's launches enqueued from its
        own host thread (rmsf_multi_push_frames; no host synchronisation).
        ``reset``: reset the state ``mode`` accumulates into first;
        ``ref_frames[i]`` / ``shift_frames[i]``: device frames set as the
        reference / merge shift frame first; ``merge_slabs``: 0 = auto (atom
        slabs from 1M atoms, run by the next multi_chan_merge), 1 = off.
        ``after_torch``: order each context stream after torch's current
        stream of the tensor's device (skip when the frames are known ready)."""
        import torch

        n = len(ctxs)
        if len(frames) != n:
            raise ValueError("one frame tensor per context")
        ptrs, counts = (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
        refs = (ctypes.c_void_p * n)() if ref_frames is not None else None
        shifts = (ctypes.c_void_p * n)() if shift_frames is not None else None
        for i, (c, t) in enumerate(zip(ctxs, frames)):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise ValueError("multi_push_frames: contiguous float32 HIP tensors expected")
            if t.numel() % (3 * c.n_atoms):
                raise ValueError(f"device frames: not a whole number of {c.n_atoms}-atom frames")
            if t.device.index != c.device:
                raise ValueError(f"context {i} is on device {c.device}, its frames on {t.device}")
            ptrs[i], counts[i] = t.data_ptr(), t.numel() // (3 * c.n_atoms)
            keep = [t]
            for arr, src in ((refs, ref_frames), (shifts, shift_frames)):
                if arr is not None and src[i] is not None:
                    f = src[i]
                    if not (f.is_cuda and f.dtype == torch.float32 and f.is_contiguous()
                            and f.numel() == 3 * c.n_atoms and f.device.index == c.device):
                        raise ValueError("reference / shift frames: one contiguous float32 frame on the "
                                         "context's device")
                    arr[i] = f.data_ptr()
                    keep.append(f)
            if after_torch:
                c._after_torch(t)
            c._alive.update((id(k), k) for k in keep)
        h, _ = Context._handles(ctxs)
        call("rmsf_multi_push_frames", h, n, ptrs, counts, 0, int(mode), RMSF_MULTI_RESET if reset else 0,
             refs, shifts, int(merge_slabs))
