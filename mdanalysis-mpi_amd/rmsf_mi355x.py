#!/usr/bin/env python3
"""Script mode: ``RMSF.py`` on MI355X.

    # RMSF.py's own run (mpirun -n P python RMSF.py) -> one process per GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29500 rmsf_mi355x.py \\
        --topology adk.gro --trajectory adk.xtc

    # without MDAnalysis: a synthetic trajectory generated in HBM
    python rmsf_mi355x.py --synthetic 100000 2000 --align frame0

Without MDAnalysis, a .gro or .psf topology and an .xtc, .dcd (or
multi-frame .gro) trajectory are read natively (rmsf_amd.topology /
rmsf_amd.xtc / rmsf_amd.dcd) and the selection is evaluated by the native
subset of the selection language (BASELINE C1: adk PSF/DCD).

Defaults mirror RMSF.py: selection "protein and name CA" (RMSF.py:77),
ref_frame 0 (RMSF.py:63), the two-sweep average alignment (RMSF.py:89-140),
frame blocks per rank (RMSF.py:65-69) with the per-rank range printed as at
RMSF.py:74, the ranks' statistics merged by a reduce to rank 0
(RMSF.py:143's ``comm.reduce(root=0)``; ``--merge all`` / ``scatter`` for the
all-reduce / the reduce-scatter by atom slices) and the RMSF computed on
rank 0 (RMSF.py:145-146) -- which this script also writes out (``--out``),
where RMSF.py only says "#Do something with RMSF" (RMSF.py:147).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def main(argv=None) -> int:
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--topology")
    ap.add_argument("--trajectory")
    ap.add_argument("--select", default="protein and name CA")
    ap.add_argument("--synthetic", nargs=2, type=int, metavar=("N_ATOMS", "N_FRAMES"))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--align", choices=["average", "frame0", "none"], default="average")
    ap.add_argument("--ref-frame", type=int, default=0)
    ap.add_argument("--out", default=None, help="write rank 0's RMSF (.npy)")
    ap.add_argument("--merge", choices=["root", "all", "scatter"], default="root",
                    help="N>1: reduce to rank 0 (RMSF.py:143, default), all-reduce, or reduce-scatter by atom slices")
    ap.add_argument("--exact", action="store_true",
                    help="with --align none: RMSF.py:120-146 with the script's own arithmetic, bit for bit "
                         "(per-frame Welford, ranks reduced by second_order_moments in comm.reduce's order)")
    ap.add_argument("--merge-order", choices=["mpi4py", "rank"], default="mpi4py",
                    help="--exact, N>1: the order RMSF.py:143's comm.reduce applies second_order_moments in "
                         "(mpi4py: its default binomial tree; rank: rank order)")
    a = ap.parse_args(argv)
    if a.exact and (a.align != "none" or a.merge == "scatter"):
        ap.error("--exact needs --align none and --merge root or all")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from rmsf_amd import RMSF, parallel
    from rmsf_amd.engine import Engine
    from rmsf_amd.pipeline import run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList
    from rmsf_amd.synth import generate, motion_table

    align = None if a.align == "none" else a.align
    rank, size = parallel.world()
    root = None if a.merge == "all" else 0
    if a.synthetic:
        n_atoms, n_frames = a.synthetic
        eng = Engine()
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        print("Process:%3d --> Frames: %10d -- %10d" % (rank, b0, b1), flush=True)
        motion = motion_table(a.seed + 1, n_frames) if align else None
        shard = generate(eng, n_atoms, b0, max(b1 - b0, 1), seed=a.seed, motion=motion)[: b1 - b0]
        res = run_pipeline(eng, DeviceSource(shard, offset=b0, n_traj=n_frames), FrameList(n_frames),
                           align=align, ref_frame=a.ref_frame, merge_root=root, merge_scatter=a.merge == "scatter",
                           exact=a.exact, merge_order=a.merge_order)
        rmsf = None if res.rmsf is None else res.rmsf.cpu().numpy()   # None on the non-root ranks
    else:
        if not (a.topology and a.trajectory):
            ap.error("--topology/--trajectory (MDAnalysis) or --synthetic is required")
        try:
            import MDAnalysis as mda
        except ImportError:
            mda = None
        if mda is not None:
            u = mda.Universe(a.topology, a.trajectory)
            ag = u.select_atoms(a.select)
            rmsf = RMSF(ag, align=align, ref_frame=a.ref_frame, verbose=True, merge_root=root,
                        merge_scatter=a.merge == "scatter", exact=a.exact,
                        merge_order=a.merge_order).run().results.rmsf
        else:
            # native fallback: GRO or PSF topology + selection subset; XTC, DCD (or
            # multi-frame GRO) trajectory.  PSF masses (GRO: masses guessed from
            # the atom names, as MDAnalysis' GROParser does) feed the
            # mass-weighted centre of mass RMSF.py uses (RMSF.py:84,94,117,127).
            from rmsf_amd.topology import GroTopology, PsfTopology

            ext = a.topology.lower().rsplit(".", 1)[-1]
            if ext not in ("gro", "psf"):
                ap.error("without MDAnalysis only .gro and .psf topologies are read natively")
            top = GroTopology(a.topology) if ext == "gro" else PsfTopology(a.topology)
            sel = top.select(a.select)
            masses = None if top.masses is None else top.masses[sel]
            traj = (a.trajectory if a.trajectory.lower().endswith((".xtc", ".dcd"))
                    else GroTopology(a.trajectory).frames)
            rmsf = RMSF(traj, select=sel, align=align, masses=masses, ref_frame=a.ref_frame,
                        verbose=True, merge_root=root, merge_scatter=a.merge == "scatter", exact=a.exact,
                        merge_order=a.merge_order).run().results.rmsf
    if rank == 0:
        print(f"RMSF over {len(rmsf)} atoms: mean {rmsf.mean():.6f} A, max {rmsf.max():.6f} A", flush=True)
        if a.out:
            np.save(a.out, rmsf)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
