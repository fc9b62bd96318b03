"""Device engine: thin typed wrappers around the C ABI on torch-allocated HBM.

torch is plumbing here (the caching allocator for HBM buffers, the current
HIP stream, torch.distributed for RCCL); every byte of arithmetic on the hot
path runs in the hand-written HIP kernels of csrc/rmsf_kernels.hip.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import RMSF_MODE_SUM, RMSF_MODE_WELFORD, RMSF_REFINFO_DOUBLES, RMSF_XFORM_DOUBLES, call

F64 = torch.float64
F32 = torch.float32


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


class Engine:
    """Launches the RMSF kernels on one device, on torch's current stream."""

    def __init__(self, device: torch.device | int | str | None = None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("rmsf_amd needs a HIP device (MI355X); none is visible -- no CPU fallback exists")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError(f"rmsf_amd runs on HIP devices only, got {self.device}")
        call("rmsf_set_device", self.device.index if self.device.index is not None else 0)

    # -- helpers -----------------------------------------------------------
    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    @property
    def side_stream(self) -> torch.cuda.Stream:
        """A second stream on the device, for work that must not queue ahead
        of the launching stream's kernels (the merge shift's gather)."""
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        return self._side

    def empty(self, *shape, dtype=F64) -> torch.Tensor:
        return torch.empty(*shape, dtype=dtype, device=self.device)

    def zeros(self, *shape, dtype=F64) -> torch.Tensor:
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def sel_tensor(self, sel) -> torch.Tensor | None:
        if sel is None:
            return None
        s = torch.as_tensor(np.ascontiguousarray(sel, dtype=np.int32)).to(self.device)
        return s

    # -- kernels -----------------------------------------------------------
    def reference_setup(self, n_sel: int, *, frame_ptr: int | None = None, avg: torch.Tensor | None = None,
                        sel: torch.Tensor | None = None, masses: torch.Tensor | None = None):
        """RMSF.py:80-87 (frame) / 113-118 (average): centred f64 reference + info."""
        ref = self.empty(n_sel, 3)
        info = self.empty(RMSF_REFINFO_DOUBLES)
        call("rmsf_reference_setup", frame_ptr, _ptr(avg), n_sel, _ptr(sel if frame_ptr else None), _ptr(masses),
             ref.data_ptr(), info.data_ptr(), self.stream)
        return ref, info

    def reference_setup_mean(self, total: torch.Tensor, n_frames: float, n_sel: int,
                             masses: torch.Tensor | None = None):
        """RMSF.py:111 + 113-118: the average total / n_frames and the
        reference from it (one launch up to 1,024 selected atoms);
        bit-identical to ``divide`` + ``reference_setup(avg=...)``."""
        avg = self.empty(3 * n_sel)
        ref = self.empty(n_sel, 3)
        info = self.empty(RMSF_REFINFO_DOUBLES)
        call("rmsf_reference_setup_mean", total.data_ptr(), float(n_frames), n_sel, _ptr(masses), avg.data_ptr(),
             ref.data_ptr(), info.data_ptr(), self.stream)
        return avg, ref, info

    def workspace_bytes(self, n_sel: int, n_frames: int) -> int:
        return int(self.lib.rmsf_superpose_workspace_bytes(n_sel, n_frames))

    def superpose(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, masses, ref, refinfo,
                  xform: torch.Tensor, work: torch.Tensor, pstride: int = 0, dense_out: int | None = None,
                  dense_stride: int = 0) -> None:
        """RMSF.py:94-97,127-131 + get_rotation_matrix (RMSF.py:43-51): per-frame COM + QCP.
        ``pstride`` > 0: frames stored as coordinate planes (rmsf_superpose_planes).
        ``dense_out`` (a gathered ``sel``): also write the selected rows to
        that device address, frame f's [n_sel, 3] at f * ``dense_stride``
        floats (0 = 3 n_sel; rmsf_superpose_compact)."""
        if dense_out is not None:
            call("rmsf_superpose_compact", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(masses),
                 ref.data_ptr(), refinfo.data_ptr(), xform.data_ptr(), work.data_ptr(),
                 work.numel() * work.element_size(), dense_out, dense_stride, self.stream)
            return
        if pstride:
            call("rmsf_superpose_planes", xyz_ptr, fstride, pstride, n_frames, n_sel, _ptr(sel), _ptr(masses),
                 ref.data_ptr(), refinfo.data_ptr(), xform.data_ptr(), work.data_ptr(),
                 work.numel() * work.element_size(), self.stream)
            return
        call("rmsf_superpose", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(masses), ref.data_ptr(),
             refinfo.data_ptr(), xform.data_ptr(), work.data_ptr(), work.numel() * work.element_size(), self.stream)

    def splits(self, n_sel: int, n_frames: int, aligned: bool) -> int:
        return int(self.lib.rmsf_accumulate_splits(n_sel, n_frames, int(aligned)))

    def split_counts(self, n_frames: int, n_splits: int) -> list[int]:
        return [int(self.lib.rmsf_split_count(n_frames, n_splits, s)) for s in range(n_splits)]

    def accumulate(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, xform, refinfo, mode: int,
                   n_splits: int, out0: torch.Tensor, out1: torch.Tensor | None) -> None:
        """RMSF.py:99-103 (SUM) / 133-138 (WELFORD) over split frame tiles."""
        call("rmsf_accumulate", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(xform), _ptr(refinfo), mode,
             n_splits, out0.data_ptr(), _ptr(out1), self.stream)

    def balanced_workspace_bytes(self, n_sel: int, n_frames: int, n_groups: int = 0) -> int:
        return int(self.lib.rmsf_accumulate_balanced_workspace_bytes(n_sel, n_frames, n_groups))

    def accumulate_balanced(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, xform, refinfo,
                            mode: int, work: torch.Tensor, n_groups: int = 0, pstride: int = 0) -> None:
        """RMSF.py:99-103 (SUM) / 133-138 (WELFORD) on the balanced grid (one equal
        (lane chunk, frame) range per workgroup); partials go to ``work``.
        ``pstride`` > 0: aligned sweep over coordinate planes read in place."""
        if pstride:
            call("rmsf_accumulate_balanced_planes", xyz_ptr, fstride, pstride, n_frames, n_sel, _ptr(sel),
                 _ptr(xform), _ptr(refinfo), mode, n_groups, work.data_ptr(), work.numel() * work.element_size(),
                 self.stream)
            return
        call("rmsf_accumulate_balanced", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(xform), _ptr(refinfo),
             mode, n_groups, work.data_ptr(), work.numel() * work.element_size(), self.stream)

    def fold_balanced(self, work: torch.Tensor, n_coord: int, mode: int, acc_n: int, acc0: torch.Tensor,
                      acc1: torch.Tensor | None) -> None:
        """Fold the balanced partials in frame order into the running result
        (Chan's merge, RMSF.py:36-41, or a sum)."""
        call("rmsf_fold_balanced", work.data_ptr(), n_coord, mode, acc_n, acc0.data_ptr(), _ptr(acc1), self.stream)

    def fold_balanced_finalize(self, work: torch.Tensor, n_coord: int, acc_n: int, acc0: torch.Tensor,
                               acc1: torch.Tensor, n_total: int, rmsf: torch.Tensor) -> None:
        """fold_balanced (WELFORD) + finalize (RMSF.py:146) in one launch, for
        an atom plan (aligned sweeps, gathered selections, planes)."""
        call("rmsf_fold_balanced_finalize", work.data_ptr(), n_coord, acc_n, acc0.data_ptr(), acc1.data_ptr(),
             n_total, rmsf.data_ptr(), self.stream)

    def fold_balanced_shift(self, work: torch.Tensor, n_coord: int, acc_n: int, acc0: torch.Tensor,
                            acc1: torch.Tensor, shift: torch.Tensor, off3, out: torch.Tensor) -> None:
        """fold_balanced (WELFORD) + chan_shift_pack in one launch: ``out`` =
        the moments about c = shift + off3 that the cross-rank merge sums."""
        if out.numel() < 2 * n_coord or shift.numel() < n_coord:
            raise ValueError("fold_balanced_shift: buffer sizes")
        call("rmsf_fold_balanced_shift", work.data_ptr(), n_coord, acc_n, acc0.data_ptr(), acc1.data_ptr(),
             shift.data_ptr(), int(shift.dtype == torch.float32), _ptr(off3), out.data_ptr(), self.stream)

    def fold_balanced_shift_sliced(self, work: torch.Tensor, n_coord: int, acc_n: int, acc0: torch.Tensor,
                                   acc1: torch.Tensor, shift: torch.Tensor, off3, slice_coords: int,
                                   out: torch.Tensor) -> None:
        """fold_balanced_shift writing the reduce-scatter merge's atom-sliced
        layout: slice r (slice_coords coordinates) as [T1 | T2] at
        out[2 r slice_coords:]."""
        n_slices = -(-n_coord // slice_coords)
        if out.numel() < 2 * slice_coords * n_slices or shift.numel() < n_coord:
            raise ValueError("fold_balanced_shift_sliced: buffer sizes")
        call("rmsf_fold_balanced_shift_sliced", work.data_ptr(), n_coord, acc_n, acc0.data_ptr(), acc1.data_ptr(),
             shift.data_ptr(), int(shift.dtype == torch.float32), _ptr(off3), slice_coords, out.data_ptr(),
             self.stream)

    def balanced_slab_chunks(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int) -> int:
        """Chunks (1024 coordinates each) of the flat balanced plan when it is
        chunk-aligned (atom slabs possible), else 0."""
        c = ctypes.c_int64(0)
        call("rmsf_balanced_slab_chunks", xyz_ptr, fstride, n_frames, n_sel, ctypes.cast(ctypes.pointer(c),
                                                                                        ctypes.c_void_p))
        return int(c.value)

    def accumulate_balanced_slab(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, c0: int, c1: int,
                                 work: torch.Tensor) -> None:
        """The whole flat plan's ranges of chunks [c0, c1) (WELFORD)."""
        call("rmsf_accumulate_balanced_slab", xyz_ptr, fstride, n_frames, n_sel, c0, c1, work.data_ptr(),
             work.numel() * work.element_size(), self.stream)

    def fold_balanced_shift_slab(self, work: torch.Tensor, n_coord: int, acc_n: int, acc0: torch.Tensor,
                                 acc1: torch.Tensor, shift: torch.Tensor, off3, out: torch.Tensor, c0: int,
                                 c1: int) -> None:
        """Fold chunks [c0, c1) and write their [T1 | T2] to ``out``."""
        j0, j1 = 1024 * c0, min(1024 * c1, n_coord)
        if out.numel() < 2 * (j1 - j0) or shift.numel() < n_coord:
            raise ValueError("fold_balanced_shift_slab: buffer sizes")
        call("rmsf_fold_balanced_shift_slab", work.data_ptr(), n_coord, acc_n, acc0.data_ptr(), acc1.data_ptr(),
             shift.data_ptr(), int(shift.dtype == torch.float32), _ptr(off3), out.data_ptr(), c0, c1, self.stream)

    def chan_merge(self, mean_parts: torch.Tensor, m2_parts: torch.Tensor, counts, n_coord: int,
                   mean_out: torch.Tensor, m2_out: torch.Tensor) -> None:
        """second_order_moments (RMSF.py:36-41) folded over the partials in order."""
        c = _lib.i64p(counts)
        call("rmsf_chan_merge", mean_parts.data_ptr(), m2_parts.data_ptr(), ctypes.cast(c, ctypes.c_void_p),
             len(counts), n_coord, mean_out.data_ptr(), m2_out.data_ptr(), self.stream)

    def chan_reduce(self, mean_parts: torch.Tensor, m2_parts: torch.Tensor, counts, n_coord: int,
                    mean_out: torch.Tensor, m2_out: torch.Tensor, order="mpi4py") -> None:
        """RMSF.py:143's comm.reduce of the partials (rank order in the rows)
        with second_order_moments in ``order`` ("mpi4py": mpi4py's default
        binomial tree; "rank": rank order).  The parts are overwritten (the
        schedule's working storage)."""
        c = _lib.i64p(counts)
        call("rmsf_chan_reduce", mean_parts.data_ptr(), m2_parts.data_ptr(), ctypes.cast(c, ctypes.c_void_p),
             len(counts), n_coord, _lib.merge_order(order), mean_out.data_ptr(), m2_out.data_ptr(), self.stream)

    def chan_merge_pair(self, mean1: torch.Tensor, m21: torch.Tensor, n1: int, mean2: torch.Tensor,
                        m22: torch.Tensor, n2: int) -> None:
        """(mean1, m21) = second_order_moments((n1, mean1, m21), (n2, mean2, m22)) in place."""
        n = mean1.numel()
        if m21.numel() != n or mean2.numel() != n or m22.numel() != n:
            raise ValueError("chan_merge_pair: buffer sizes")
        call("rmsf_chan_merge_pair", mean1.data_ptr(), m21.data_ptr(), int(n1), mean2.data_ptr(), m22.data_ptr(),
             int(n2), n, self.stream)

    def sum_splits(self, parts: torch.Tensor, n_parts: int, n: int, out: torch.Tensor) -> None:
        call("rmsf_sum_splits", parts.data_ptr(), n_parts, n, out.data_ptr(), self.stream)

    def divide(self, x: torch.Tensor, divisor: float, out: torch.Tensor) -> None:
        call("rmsf_divide", x.data_ptr(), float(divisor), x.numel(), out.data_ptr(), self.stream)

    def chan_weight(self, mean_k: torch.Tensor, w: float, out: torch.Tensor) -> None:
        call("rmsf_chan_weight", mean_k.data_ptr(), float(w), mean_k.numel(), out.data_ptr(), self.stream)

    def chan_deviation(self, mean_k, m2_k, mean, n_k: float, out) -> None:
        call("rmsf_chan_deviation", mean_k.data_ptr(), m2_k.data_ptr(), mean.data_ptr(), float(n_k), mean_k.numel(),
             out.data_ptr(), self.stream)

    def chan_shift_pack(self, mean_k, m2_k, shift, off3, n_k: float, out) -> None:
        """out[0:n] = n_k (mean_k - c), out[n:2n] = M2_k + n_k (mean_k - c)^2,
        c = shift + off3 (per xyz); shift f64 or f32."""
        n = mean_k.numel()
        if out.numel() < 2 * n or shift.numel() < n:
            raise ValueError("chan_shift_pack: buffer sizes")
        call("rmsf_chan_shift_pack", mean_k.data_ptr(), m2_k.data_ptr(), shift.data_ptr(),
             int(shift.dtype == torch.float32), _ptr(off3), float(n_k), n, out.data_ptr(), self.stream)

    def chan_shift_finish(self, t, shift, off3, n_sel: int, n_frames: int, mean, m2, rmsf) -> None:
        if t.numel() < 6 * n_sel or shift.numel() < 3 * n_sel or mean.numel() < 3 * n_sel or m2.numel() < 3 * n_sel:
            raise ValueError("chan_shift_finish: buffer sizes")
        call("rmsf_chan_shift_finish", t.data_ptr(), shift.data_ptr(), int(shift.dtype == torch.float32), _ptr(off3),
             n_sel, n_frames, mean.data_ptr(), m2.data_ptr(), _ptr(rmsf), self.stream)

    def chan_shift_pack_sliced(self, mean_k, m2_k, shift, off3, n_k: float, slice_coords: int, out) -> None:
        """chan_shift_pack into the atom-sliced layout (see
        fold_balanced_shift_sliced)."""
        n = mean_k.numel()
        if out.numel() < 2 * slice_coords * -(-n // slice_coords) or shift.numel() < n:
            raise ValueError("chan_shift_pack_sliced: buffer sizes")
        call("rmsf_chan_shift_pack_sliced", mean_k.data_ptr(), m2_k.data_ptr(), shift.data_ptr(),
             int(shift.dtype == torch.float32), _ptr(off3), float(n_k), n, slice_coords, out.data_ptr(), self.stream)

    def chan_shift_finish_slice(self, t, slice_coords: int, shift, off3, n_sel: int, n_frames: int, mean, m2,
                                rmsf) -> None:
        """Unpack one reduced slice [T1 | T2] (width slice_coords) for its
        n_sel atoms; shift / mean / m2 / rmsf start at the slice's first atom."""
        if (t.numel() < 2 * slice_coords or 3 * n_sel > slice_coords or shift.numel() < 3 * n_sel
                or mean.numel() < 3 * n_sel or m2.numel() < 3 * n_sel):
            raise ValueError("chan_shift_finish_slice: buffer sizes")
        call("rmsf_chan_shift_finish_slice", t.data_ptr(), slice_coords, shift.data_ptr(),
             int(shift.dtype == torch.float32), _ptr(off3), n_sel, n_frames, mean.data_ptr(), m2.data_ptr(),
             _ptr(rmsf), self.stream)

    def zero_index(self) -> torch.Tensor:
        """A resident int64 [0] (row index for gathering one frame); made once."""
        if getattr(self, "_zero_idx", None) is None:
            self._zero_idx = torch.zeros(1, dtype=torch.int64, device=self.device)
        return self._zero_idx

    def gather_frames(self, base_ptr: int, fstride: int, rows: torch.Tensor, n: int, n_sel: int, sel,
                      out: torch.Tensor) -> None:
        """out[i] = frame base + rows[i]*fstride, selected (rmsf_gather_frames)."""
        if out.dtype != F32 or out.numel() < 3 * n_sel * n or rows.numel() < n:
            raise ValueError("gather_frames: buffer sizes")
        call("rmsf_gather_frames", base_ptr, fstride, rows.data_ptr(), n, n_sel, _ptr(sel), out.data_ptr(),
             self.stream)

    def planes_to_rows(self, x: torch.Tensor, n: int) -> torch.Tensor:
        """f64 [3n] in plane order (x[n], y[n], z[n]) -> a new [3n] in (atom, xyz) order."""
        out = self.empty(3 * n)
        call("rmsf_planes_to_rows", x.data_ptr(), n, out.data_ptr(), self.stream)
        return out

    def welford_sequential(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, k0: int,
                           mean: torch.Tensor, sumsquares: torch.Tensor,
                           work: torch.Tensor | None = None) -> torch.Tensor:
        """RMSF.py:137-138 as written, frame by frame from k = k0 (k0 = 0:
        the state starts at np.zeros): the reference recurrence's own
        (mean, sumsquares), bit for bit.  Unaligned rows; ``sel`` an int32
        device index tensor or None.  Returns the coefficient workspace
        (pass it back to reuse it)."""
        need = int(self.lib.rmsf_welford_sequential_workspace_bytes(n_frames))
        if work is None or work.numel() * work.element_size() < need:
            work = self.empty(max(need, 16) // 8)
        call("rmsf_welford_sequential", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), k0, mean.data_ptr(),
             sumsquares.data_ptr(), work.data_ptr(), work.numel() * work.element_size(), self.stream)
        return work

    # -- exact=True on the aligned path (the reference's summation orders) ---
    def reference_setup_seq(self, n_sel: int, mass_total: float, *, frame_ptr: int | None = None,
                            sel: torch.Tensor | None = None, total: torch.Tensor | None = None,
                            n_frames: float = 1.0, masses: torch.Tensor | None = None, after_centre=None):
        """RMSF.py:84-85 (``frame_ptr``) or RMSF.py:111 + 117-118 (``total``,
        the all-reduced sweep-1 sums, divided by ``n_frames`` as read) with
        the reference's own summation order (rmsf_reference_setup_sequential).
        ``after_centre``: called between the two halves (the centred
        reference, then the record's sums; rmsf_reference_centre_sequential /
        rmsf_reference_sums_sequential, same bits) -- e.g. to record an event
        an InnerProduct on another stream waits for.  Returns (average or
        None, ref, info)."""
        ref = self.empty(n_sel, 3)
        info = self.empty(RMSF_REFINFO_DOUBLES)
        avg = self.empty(3 * n_sel) if total is not None else None
        args = (frame_ptr, _ptr(total), float(n_frames), n_sel, _ptr(sel if frame_ptr else None), _ptr(masses),
                float(mass_total), _ptr(avg), ref.data_ptr(), info.data_ptr(), self.stream)
        if after_centre is None:
            call("rmsf_reference_setup_sequential", *args)
        else:
            call("rmsf_reference_centre_sequential", *args)
            after_centre()
            call("rmsf_reference_sums_sequential", n_sel, float(mass_total), ref.data_ptr(), info.data_ptr(),
                 self.stream)
        return avg, ref, info

    def superpose_seq(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, masses,
                      mass_total: float, ref: torch.Tensor, refinfo: torch.Tensor, xform: torch.Tensor) -> None:
        """RMSF.py:94-97,127-131 + get_rotation_matrix per frame in the
        reference's order (rmsf_superpose_sequential)."""
        call("rmsf_superpose_sequential", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(masses),
             float(mass_total), ref.data_ptr(), refinfo.data_ptr(), xform.data_ptr(), self.stream)

    def frame_com_seq(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, masses,
                      mass_total: float, xform: torch.Tensor) -> None:
        """The first half of superpose_seq: every frame's mobile COM into the
        records' [9..11] (rmsf_frame_com_sequential); no reference needed."""
        call("rmsf_frame_com_sequential", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(masses),
             float(mass_total), xform.data_ptr(), self.stream)

    def superpose_seq_from_com(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel,
                               ref: torch.Tensor, refinfo: torch.Tensor, xform: torch.Tensor) -> None:
        """The second half: InnerProduct + QCP from the COMs in the records
        (rmsf_superpose_sequential_from_com)."""
        call("rmsf_superpose_sequential_from_com", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), ref.data_ptr(),
             refinfo.data_ptr(), xform.data_ptr(), self.stream)

    def inner_product_seq(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, ref: torch.Tensor,
                          xform: torch.Tensor) -> None:
        """superpose_seq_from_com's first part: qcprot's InnerProduct per
        frame against the centred reference (rmsf_inner_product_sequential;
        the record's sums need not be ready)."""
        call("rmsf_inner_product_sequential", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), ref.data_ptr(),
             xform.data_ptr(), self.stream)

    def superpose_seq_qcp(self, n_frames: int, n_sel: int, refinfo: torch.Tensor, xform: torch.Tensor) -> None:
        """Its second part: E0 with the record's G2, and the QCP
        (rmsf_superpose_sequential_qcp)."""
        call("rmsf_superpose_sequential_qcp", n_frames, n_sel, refinfo.data_ptr(), xform.data_ptr(), self.stream)

    def accumulate_seq(self, xyz_ptr: int, fstride: int, n_frames: int, n_sel: int, sel, xform, refinfo,
                       mode: int, k0: int, acc0: torch.Tensor, acc1: torch.Tensor | None,
                       work: torch.Tensor | None = None) -> torch.Tensor | None:
        """RMSF.py:99-103 (SUM) / 133-138 (WELFORD) frame by frame in order
        (rmsf_accumulate_sequential); returns the coefficient workspace."""
        if mode == RMSF_MODE_WELFORD:
            need = int(self.lib.rmsf_welford_sequential_workspace_bytes(n_frames))
            if work is None or work.numel() * work.element_size() < need:
                work = self.empty(max(need, 16) // 8)
        call("rmsf_accumulate_sequential", xyz_ptr, fstride, n_frames, n_sel, _ptr(sel), _ptr(xform),
             _ptr(refinfo), mode, k0, acc0.data_ptr(), _ptr(acc1), _ptr(work),
             0 if work is None else work.numel() * work.element_size(), self.stream)
        return work

    def finalize(self, m2: torch.Tensor, n_sel: int, n_frames: int, out: torch.Tensor) -> None:
        """RMSF.py:146: sqrt(M2.sum(axis=1)/n)."""
        call("rmsf_finalize", m2.data_ptr(), n_sel, n_frames, out.data_ptr(), self.stream)

    def qcp_batch(self, A: torch.Tensor, E0: torch.Tensor, N: torch.Tensor):
        n = A.shape[0]
        rot = self.empty(n, 9)
        rmsd = self.empty(n)
        call("rmsf_qcp_batch", A.data_ptr(), E0.data_ptr(), N.data_ptr(), n, rot.data_ptr(), rmsd.data_ptr(),
             self.stream)
        return rot, rmsd

    def synth_frames(self, out: torch.Tensor, n_atoms: int, f0: int, nf: int, seed: int,
                     motion: torch.Tensor | None = None, fstride: int | None = None) -> None:
        fstride = 3 * n_atoms if fstride is None else fstride
        call("rmsf_synth_frames", out.data_ptr(), fstride, n_atoms, f0, nf, ctypes.c_uint64(seed).value,
             _ptr(motion), self.stream)


def block_range(n_frames: int, size: int, rank: int) -> tuple[int, int]:
    """RMSF.py:63-72 through the C ABI (bit-exact integer arithmetic)."""
    a, b = ctypes.c_int64(), ctypes.c_int64()
    call("rmsf_block_range", n_frames, size, rank, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


__all__ = ["Engine", "block_range", "RMSF_MODE_SUM", "RMSF_MODE_WELFORD", "RMSF_XFORM_DOUBLES"]
