"""``RMSF`` -- drop-in for ``MDAnalysis.analysis.rms.RMSF`` on MI355X.

The reference (RMSF.py:1-18) states its workflow as::

    average = align.AverageStructure(u, u, select='protein and name CA', ref_frame=0).run()
    aligner = align.AlignTraj(u, average.results.universe, select='protein and name CA', in_memory=True).run()
    R = rms.RMSF(c_alphas).run()            # -> R.results.rmsf

and implements it with mpi4py frame blocks.  ``RMSF(ag, align="average")``
computes exactly that (the two sweeps of RMSF.py:89-140), ``align=None`` is
plain ``rms.RMSF`` on an already-aligned trajectory, and ``align="frame0"``
superposes every frame on ``ref_frame`` first (config C3).  Under
``torch.distributed`` (one process per GPU) the frames are split into the
contiguous blocks of RMSF.py:65-69 and merged with RCCL.

Inputs: an MDAnalysis AtomGroup, a host ``numpy`` float32 array
[n_frames, n_atoms, 3] (or [n_frames, 3, n_atoms] coordinate planes with
``layout="soa"``), an HBM-resident torch tensor [n_frames, n_atoms, 3], or the
path of a GROMACS ``.xtc`` or CHARMM/NAMD ``.dcd`` file (read natively,
selection by ``select``).

``run(start, stop, step)`` or ``run(frames=...)`` (indices or a boolean mask,
as ``AnalysisBase.run``; taken in ascending order, so ``results.rmsd`` with
``collect_rmsd=True`` follows the sorted frames).

``collect_transforms=True`` (aligned runs, one device per process) adds
``results.transforms`` -- f64 [n_local, 16] per-frame records of the last
sweep: the rotation of RMSF.py:48-51 row-major in 0..8, the mobile centre of
mass of RMSF.py:94 in 9..11, the QCP rmsd in 12 -- and, for
``align="average"``, ``results.transforms_sweep1`` for RMSF.py's first sweep.
"""
from __future__ import annotations

import numpy as np
import torch

from . import parallel
from .engine import Engine
from .pipeline import run_pipeline
from .sources import AtomGroupSource, DcdSource, DeviceSource, FrameList, HostSource, XtcSource


class Results(dict):
    """Attribute-access dict, like ``MDAnalysis.analysis.base.Results``."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class RMSF:
    """Per-atom root-mean-square fluctuation, ``results.rmsf`` (f64 [n_sel]).

    Parameters
    ----------
    atomgroup : MDAnalysis AtomGroup | np.ndarray | torch.Tensor
        The selection to analyse, or a float32 trajectory [F, n_atoms, 3].
    select : array of int, optional
        Atom indices (array inputs only); default all atoms.
    align : None | "frame0" | "average"
        Superposition before the statistics (see module docstring).
    masses : array, optional
        Per-selected-atom masses for the centre of mass (RMSF.py:84,94 use
        ``center_of_mass``); default uniform.  For an AtomGroup the group's
        masses are used.
    ref_frame : int
        Trajectory frame of the first reference (RMSF.py:63).
    layout : "fac" | "soa"
        Array inputs: "fac" = [F, n_atoms, 3] (MDAnalysis' positions per
        frame), "soa" = [F, 3, n_atoms] (x, y and z coordinate planes per
        frame).  Host planes are interleaved by the stager on the host (the
        device path is unchanged); HBM-resident planes are gathered into
        (frame, atom, xyz) batches on the device (rmsf_gather_planes).
    merge_root : int, optional
        Under ``torch.distributed``: merge the ranks' statistics with a
        reduce to this rank only, as RMSF.py:143 (``comm.reduce(root=0)``)
        does; the other ranks' ``results.rmsf`` / ``mean`` / ``sumsquares``
        are None.  Default: every rank receives the merged result.  With
        ``gpus=``: the merge is a reduce to that device index and the
        results (which this one process returns either way) come from it.
    merge_scatter : bool
        Under ``torch.distributed``: merge by a reduce-scatter of atom slices
        instead -- each rank finishes its slice and only the RMSF is gathered
        to ``merge_root`` (default 0).  ``results.rmsf`` on that rank; every
        rank's ``results.atom_slice``, ``slice_mean`` and
        ``slice_sumsquares`` hold its slice (``mean``/``sumsquares`` are
        None).
    exact : bool | None
        True: compute RMSF.py with the reference's own arithmetic and
        summation orders, so ``results`` are bit-identical to the script's
        on the same float32 coordinates (``mean``, ``sumsquares``, ``rmsf``
        and, aligned, ``average``, ``rmsd`` and ``transforms``).
        align=None: RMSF.py:120-146, each rank's frames through the
        per-frame Welford of RMSF.py:137-138 in order
        (rmsf_welford_sequential) -- about 1.1-1.15x the default path's time
        on all-atom rows, by box, and about 1.0x over large gathered
        selections (``modes.c2_exact`` of BENCH_r05 and
        profiles/r06_final_tree).  Aligned:
        RMSF.py:80-146, the references, every frame's COM and qcprot inner
        product atom by atom, the sweep-1 sum and Welford frame by frame
        (the rmsf_*_sequential kernels) -- each sum an in-order add chain
        over the atoms, so its cost grows with the selection, not the
        frames: about the default's cost at RMSF.py's 214 atoms, 1.0-1.9 ms
        against 0.16-0.29 ms at 100k atoms x 100 frames (DESIGN section 5,
        "Few frames").  The ranks are
        folded by second_order_moments in RMSF.py:143's reduce order
        (``merge_order``), then RMSF.py:146.  False: the frame-parallel
        path, which agrees to ~1e-13 unaligned and, aligned, to within one
        f32 rounding flip of an aligned coordinate -- at most ulp(x) /
        sqrt(n_frames), i.e. < 1e-6 A from ~234 frames.  None (default):
        exact for aligned runs of fewer than 256 frames
        (pipeline.AUTO_EXACT_FRAMES), the frame-parallel path otherwise.
    merge_order : "mpi4py" | "rank"
        ``exact=True`` with several ranks or devices: the order in which
        RMSF.py:143's ``comm.reduce(S, op=second_order_moments)`` applies
        the op.  "mpi4py" (default): mpi4py's default object reduce
        (``rc.fast_reduce``), a binomial tree -- at 4 ranks
        op(op(S0, S1), op(S2, S3)) -- run point to point as mpi4py runs it;
        "rank": op folded in rank order (``rc.fast_reduce = False``).  The
        two agree up to 3 ranks and differ in the last bits from 4.  mpi4py
        is upstream and absent here: its tree is restated from its published
        source, not verified, so from 4 ranks the bit-for-bit claim rests on
        that restatement (parity unpinned there).
    gpus : int | list of int, optional
        Drive this many devices (or these device ids) from one process: each
        takes the RMSF.py:65-69 block of its index and the blocks merge over
        RCCL (``ncclCommInitAll``).  Inputs: host array, ``.xtc``/``.dcd``
        path, AtomGroup, or HBM-resident shards -- a list of float32 HIP
        tensors, one per device, whose concatenation is the trajectory (each
        device then takes the frames it holds).  Leave unset under
        ``torch.distributed``.
    """

    def __init__(self, atomgroup, *, select=None, align=None, masses=None, ref_frame: int = 0,
                 device=None, batch_frames: int | None = None, n_splits: int | None = None,
                 collect_rmsd: bool = False, verbose: bool = False, gpus=None,
                 collect_transforms: bool = False, layout: str = "fac", merge_root: int | None = None,
                 merge_scatter: bool = False, exact: bool | None = None, merge_order: str = "mpi4py", **kwargs):
        if layout not in ("fac", "soa"):
            raise ValueError(f"layout must be 'fac' or 'soa', got {layout!r}")
        if layout == "soa" and not (isinstance(atomgroup, np.ndarray) or isinstance(atomgroup, torch.Tensor)):
            raise ValueError("layout='soa' describes a numpy array or HIP tensor [F, 3, n_atoms]; files and "
                             "AtomGroups have their own layout")
        self.layout = layout
        self.merge_root = merge_root
        self.merge_scatter = bool(merge_scatter)
        self.exact = None if exact is None else bool(exact)
        from ._lib import merge_order as _order
        _order(merge_order)
        self.merge_order = merge_order
        self._input = atomgroup
        self.select = select
        self.align = align
        self.masses = masses
        self.ref_frame = ref_frame
        self.device = device
        self.batch_frames = batch_frames
        self.n_splits = n_splits
        self.collect_rmsd = collect_rmsd
        self.collect_transforms = collect_transforms
        self.verbose = verbose
        self.gpus = gpus
        self.results = Results()
        self._source = None

    # MDAnalysis AnalysisBase compatible signature
    def run(self, start=None, stop=None, step=None, frames=None, verbose=None, **kwargs):
        if self.gpus is not None or isinstance(self._input, (list, tuple)):
            if self.collect_transforms:
                raise NotImplementedError("collect_transforms is for one device per process")
            if self.merge_scatter:
                raise NotImplementedError("merge_scatter is for one process per GPU (torch.distributed); with "
                                          "gpus= the one process receives the merged result")
            return self._run_multi(start, stop, step, frames)  # several devices, or HBM shards per device
        eng = Engine(self.device)
        # torch's current device = the engine's, so the buffers sources and
        # caches allocate live on the device the kernels run on
        with torch.cuda.device(eng.device):
            src, masses = self._make_source(eng)
            # frames: explicit indices or a boolean mask (AnalysisBase.run(frames=...))
            fl = FrameList(src.n_traj, start, stop, step, frames=frames)
            rank, size = parallel.world()
            if verbose if verbose is not None else self.verbose:
                b0, b1 = parallel.blocks(len(fl), size)[rank]
                print("Process:%3d --> Frames: %10d -- %10d" % (rank, b0, b1))  # RMSF.py:74
            res = run_pipeline(eng, src, fl, align=self.align, masses=masses, ref_frame=self.ref_frame,
                               max_batch=self.batch_frames, n_splits=self.n_splits, collect_rmsd=self.collect_rmsd,
                               collect_transforms=self.collect_transforms, merge_root=self.merge_root,
                               merge_scatter=self.merge_scatter, exact=self.exact, merge_order=self.merge_order)
            torch.cuda.current_stream(eng.device).synchronize()
            r = self.results
            host = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731  (None: a non-root rank)
            r.rmsf = host(res.rmsf)
            r.mean = host(res.mean)
            r.sumsquares = host(res.m2)
            r.m2 = r.sumsquares
            r.n_frames = res.n_frames
            r.n_local = res.n_local
            r.block = res.block
            if res.average is not None:
                r.average = res.average.cpu().numpy()
            if res.rmsd is not None:
                r.rmsd = res.rmsd.cpu().numpy()
            if res.transforms is not None:
                r.transforms = res.transforms.cpu().numpy()
            if res.transforms_sweep1 is not None:
                r.transforms_sweep1 = res.transforms_sweep1.cpu().numpy()
            if "atom_slice" in res.extras:  # merge_scatter: this rank's slice of the statistics
                r.atom_slice = res.extras["atom_slice"]
                r.slice_mean = res.extras["slice_mean"].cpu().numpy()
                r.slice_sumsquares = res.extras["slice_m2"].cpu().numpy()
        self.n_frames = res.n_frames
        return self

    def _run_multi(self, start, stop, step, frames=None):
        """``gpus=N`` (or a list of device ids): one process drives N devices
        through the context ABI, RCCL communicators from ncclCommInitAll
        (rmsf_amd.multi)."""
        from .multi import run_multi

        out = run_multi(self._input, self.gpus, select=self.select, align=self.align, masses=self.masses,
                        ref_frame=self.ref_frame, start=start, stop=stop, step=step,
                        batch_frames=self.batch_frames, frames=frames, collect_rmsd=self.collect_rmsd,
                        layout=self.layout, merge_root=self.merge_root, exact=self.exact,
                        merge_order=self.merge_order)
        r = self.results
        r.update(out)
        r.m2 = r.sumsquares
        self.n_frames = r.n_frames
        return self

    @property
    def rmsf(self):
        return self.results.rmsf

    def _make_source(self, eng: Engine):
        x = self._input
        if hasattr(x, "batches") and hasattr(x, "reference") and hasattr(x, "n_sel"):
            return x, self.masses  # a frame source (DeviceSource, HostSource, XtcSource, ...)
        if isinstance(x, torch.Tensor):
            if x.device.type != "cuda":
                x = x.detach().cpu().numpy()
            else:
                return DeviceSource(x, self.select, layout=self.layout), self.masses
        # RMSF.py's two sweeps (align="average") read every frame twice
        # (RMSF.py:92,124): host sources then keep the staged frames in HBM
        two = self.align == "average"
        if isinstance(x, np.ndarray):
            return HostSource(x, self.select, batch_frames=self.batch_frames, cache=two,
                              layout=self.layout), self.masses
        if isinstance(x, (str, bytes)) or hasattr(x, "__fspath__"):
            import os
            path = os.fspath(x)
            if str(path).lower().endswith(".dcd"):
                # DCD frames are raw float32 planes: each batch's selected rows are
                # read from the memory-mapped file and streamed through the stager
                return DcdSource(path, self.select, batch_frames=self.batch_frames, cache=two), self.masses
            if not str(path).lower().endswith(".xtc"):
                raise ValueError(f"only .xtc and .dcd trajectory files are read natively, got {path!r}")
            # aligned runs read the reference frame first (and RMSF.py's two sweeps read
            # every frame twice): keep the decoded frames resident in HBM
            return XtcSource(path, self.select, batch_frames=self.batch_frames,
                             cache=self.align is not None), self.masses
        if hasattr(x, "universe") and hasattr(x, "positions"):
            masses = self.masses
            if masses is None and self.align is not None:
                masses = np.asarray(x.masses, dtype=np.float64)
            return AtomGroupSource(x, batch_frames=self.batch_frames, cache=two), masses
        raise TypeError(f"unsupported input {type(x)!r}: AtomGroup, numpy array or HIP torch tensor expected")
