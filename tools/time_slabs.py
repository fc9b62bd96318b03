#!/usr/bin/env python3
"""Device time of the last sweep cut into G atom slabs (pipeline.slab_sweep's
launch sequence a slab-cut merge would need: per slab the balanced
accumulate + fold) against one whole launch, on one GPU, at the strong-scaling shares of 100k x 20k frames
(20k/N frames per GPU) and C4's 1M x 2.5k share.  The slab cut is what lets
the N>1 exchanges start early (each slab's all-reduces beside the next
slab's kernels); this measures what the cut itself costs on the device
(launch boundaries, smaller grids) -- ~16 us per extra slab at 100k atoms,
more than the exchange time a cut could hide, so the pipeline does not cut.

Round 3 (``--chunk-slabs``): the pipeline's merge slabs at N > 1 -- ranges of
chunks of the WHOLE flat plan (rmsf_accumulate_balanced_slab + the slab fold
that packs T1/T2), bit-identical to the whole launch -- at C4's share,
1M atoms x 2,500 frames: the device cost of 1 / 2 / 4 / 8 slabs without the
collective (what the overlap must win back).

  python tools/time_slabs.py [--reps 20] [--chunk-slabs]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import Accumulator  # noqa: E402
from rmsf_amd.sources import Batch  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def slab_ranges(n_sel, g, align=256):
    edges = [0] + [n_sel * i // g // align * align for i in range(1, g)] + [n_sel]
    return list(zip(edges, edges[1:]))


def _slab_batch(b, a0, a1):
    return Batch(b.ptr + 12 * a0, b.fstride, b.n_frames, None)


def chunk_slabs(eng, reps):
    from rmsf_amd.pipeline import _slab_bounds
    n_atoms, nf = 1_000_000, 2_500
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    torch.cuda.synchronize()
    b = Batch(traj.data_ptr(), traj.stride(0), nf, None)
    n_chunks = eng.balanced_slab_chunks(b.ptr, b.fstride, nf, n_atoms)
    shift = traj[0].reshape(-1).clone()
    acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
    n_coord = 3 * n_atoms
    t_all = torch.empty(2 * n_coord, dtype=torch.float64, device=eng.device)
    row = {"n_atoms": n_atoms, "frames": nf, "chunks": n_chunks}
    ref = None
    for k in (1, 2, 4, 8, 1):
        slabs = _slab_bounds(n_chunks, k) if k > 1 else None
        ts_ = [torch.empty(2 * (min(1024 * c1, n_coord) - 1024 * c0), dtype=torch.float64, device=eng.device)
               for c0, c1 in (slabs or [])]

        def once():
            if slabs is None:
                eng.accumulate_balanced(b.ptr, b.fstride, nf, n_atoms, None, None, None, RMSF_MODE_WELFORD, acc.work)
                eng.fold_balanced_shift(acc.work, n_coord, 0, acc.parts0[0], acc.parts1[0], shift, None, t_all)
                return [t_all]
            for (c0, c1), t in zip(slabs, ts_):
                eng.accumulate_balanced_slab(b.ptr, b.fstride, nf, n_atoms, c0, c1, acc.work)
                eng.fold_balanced_shift_slab(acc.work, n_coord, 0, acc.parts0[0], acc.parts1[0], shift, None, t,
                                             c0, c1)
            return ts_
        out = once()
        torch.cuda.synchronize()
        flat = torch.cat([torch.cat([t[: t.numel() // 2] for t in out]), torch.cat([t[t.numel() // 2:] for t in out])])
        if ref is None:
            ref = flat.clone()
        row[f"slabs{k}_bitwise_equal_whole"] = bool(torch.equal(ref, flat))
        for _ in range(3):
            once()
        tl = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            once()
            e1.record()
            torch.cuda.synchronize()
            tl.append(e0.elapsed_time(e1))
        tl.sort()
        row[f"slabs{k}_ms_median"] = tl[len(tl) // 2]
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--chunk-slabs", action="store_true")
    a = ap.parse_args()
    eng = Engine(torch.device("cuda", 0))
    if a.chunk_slabs:
        chunk_slabs(eng, a.reps)
        return
    for n_atoms, frames_list in ((100_000, (2_500, 5_000, 10_000, 20_000)), (1_000_000, (2_500,))):
        traj = generate(eng, n_atoms, 0, max(frames_list), seed=0)
        torch.cuda.synchronize()
        for nf in frames_list:
            b = Batch(traj.data_ptr(), traj.stride(0), nf, None)
            row = {"n_atoms": n_atoms, "frames": nf}
            for g, key in ((1, "G1"), (2, "G2"), (4, "G4"), (8, "G8"), (1, "G1b")):
                slabs = slab_ranges(n_atoms, g)
                accs = [Accumulator(eng, a1 - a0, RMSF_MODE_WELFORD, nf, False) for a0, a1 in slabs]

                def once():
                    for acc, (a0, a1) in zip(accs, slabs):
                        acc.n = 0
                        acc.add(_slab_batch(b, a0, a1))
                for _ in range(3):
                    once()
                ts = []
                for _ in range(a.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    once()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                ts.sort()
                row[f"{key}_ms_median"] = ts[len(ts) // 2]
                row[f"{key}_ms_min"] = ts[0]
            print(json.dumps(row), flush=True)
        del traj
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
