#!/usr/bin/env python3
"""Aligned sweep with the superposition of batch k+1 running beside the
accumulate of batch k on a second HIP stream, against today's one-batch
two-pass sweep (RMSF.py:91-103 / 123-138: superpose, then transform +
accumulate).  Both passes are HBM streams of the same bytes; the accumulate
is VALU-heavy (45 fp64 ops per atom-frame), the superposition sums are not,
so two concurrent kernels can keep HBM busier than either alone.

Prints, per form, the median ms of the whole aligned sweep (C3: frame 0
reference, Welford) and the RMSF's max |diff| against the one-batch sweep.
python tools/ab_overlap.py [n_atoms n_frames]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD, RMSF_XFORM_DOUBLES  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import Accumulator, reference_from_frame, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def main():
    n_atoms = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000
    eng = Engine()
    traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    src = DeviceSource(traj)
    fl = FrameList(nf)
    fstride = src.fstride
    torch.cuda.synchronize()

    def base():
        return run_pipeline(eng, src, fl, align="frame0").rmsf

    ref, info = reference_from_frame(eng, src, 0, n_atoms, None)
    xf = eng.empty(nf, RMSF_XFORM_DOUBLES)
    side = torch.cuda.Stream(eng.device)

    def batched(K, overlap, lead=None, ag=0):
        bounds = [(k * nf // K, (k + 1) * nf // K) for k in range(K)]
        mb = max(b - a for a, b in bounds)
        acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, mb, True)
        need = max(eng.balanced_workspace_bytes(n_atoms, b - a, ag) for a, b in bounds)
        if need > acc.work.numel() * 8:
            acc.work = eng.empty((need + 7) // 8)
        swork = eng.empty(max(1, (max(eng.workspace_bytes(n_atoms, b - a) for a, b in bounds) + 7) // 8))
        main = torch.cuda.current_stream(eng.device)
        evs = [torch.cuda.Event() for _ in range(K)]
        done = [torch.cuda.Event() for _ in range(K)]
        sup_stream = side if overlap else main
        sup_stream.wait_stream(main)

        def sup(k):
            a, b = bounds[k]
            with torch.cuda.stream(sup_stream):
                if lead is not None and k - lead >= 0:
                    sup_stream.wait_event(done[k - lead])  # at most `lead` batches ahead
                eng.superpose(traj.data_ptr() + a * fstride * 4, fstride, b - a, n_atoms, None, None, ref, info,
                              xf[a:b], swork)
                evs[k].record(sup_stream)

        if lead is None:
            for k in range(K):
                sup(k)
        else:
            for k in range(min(K, lead)):
                sup(k)
        for k in range(K):
            a, b = bounds[k]
            main.wait_event(evs[k])
            eng.accumulate_balanced(traj.data_ptr() + a * fstride * 4, fstride, b - a, n_atoms, None, xf[a:b], info,
                                    RMSF_MODE_WELFORD, acc.work, ag)
            eng.fold_balanced(acc.work, 3 * n_atoms, RMSF_MODE_WELFORD, acc.n, acc.parts0[0], acc.parts1[0])
            acc.n += b - a
            done[k].record(main)
            if lead is not None and k + lead < K:
                sup(k + lead)
        main.wait_stream(sup_stream)
        out = eng.empty(n_atoms)
        eng.finalize(acc.result1, n_atoms, nf, out)
        return out

    def timeit(fn, reps=7):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[len(ts) // 2], r

    forms = [("one batch (today)", base)]
    for K in (2, 4, 8):
        forms.append((f"K={K} serial", lambda K=K: batched(K, False)))
        for ag in (0, 256, 512, 1024):
            forms.append((f"K={K} overlap ag={ag}", lambda K=K, ag=ag: batched(K, True, None, ag)))
    r0 = None
    print(f"aligned sweep (frame 0, Welford), {n_atoms} atoms x {nf} frames", flush=True)
    for rnd in range(2):  # two rounds, A/B order effects visible
        for name, fn in forms:
            ms, r = timeit(fn)
            if r0 is None:
                r0 = r.clone()
            d = float((r - r0).abs().max())
            print(f"  round {rnd} {name:24s} {ms:8.3f} ms   max|rmsf - one batch| {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
