#!/usr/bin/env python3
"""Config C1 shape (3341 atoms, 214 selected, 98 frames, RMSF.py's two
sweeps) replayed as a hipGraph N times, for a per-kernel breakdown under
rocprofv3 --kernel-trace --stats, or A/B of two library builds in
alternating processes.  python tools/c1_kernels.py [reps] [--lib PATH]"""
import ctypes
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd import _lib  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import CapturedPipeline, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def main():
    args = sys.argv[1:]
    if "--lib" in args:
        i = args.index("--lib")
        _lib.LIB_PATH = os.path.abspath(args[i + 1])
        del args[i:i + 2]
        old = ctypes.CDLL(_lib.LIB_PATH)
        if not hasattr(old, "rmsf_reference_setup_mean"):  # an older build: divide + setup, as it ran then
            del _lib.SIGNATURES["rmsf_reference_setup_mean"]

            def setup_mean(eng, total, n, n_sel, masses=None):
                avg = eng.empty(3 * n_sel)
                eng.divide(total, n, avg)
                return (avg, *eng.reference_setup(n_sel, avg=avg, masses=masses))

            Engine.reference_setup_mean = setup_mean
        if not hasattr(old, "rmsf_fold_balanced_finalize"):  # fold, then finalise
            del _lib.SIGNATURES["rmsf_fold_balanced_finalize"]

            def fold_finalize(eng, work, n_coord, acc_n, acc0, acc1, n_total, rmsf):
                eng.fold_balanced(work, n_coord, _lib.RMSF_MODE_WELFORD, acc_n, acc0, acc1)
                eng.finalize(acc1, n_coord // 3, n_total, rmsf)

            Engine.fold_balanced_finalize = fold_finalize
    reps = int(args[0]) if args else 200
    eng = Engine()
    n_atoms, nf = 3341, 98
    sel = np.sort(np.random.default_rng(12).choice(n_atoms, 214, replace=False))
    traj = generate(eng, n_atoms, 0, nf, seed=11, motion=motion_table(13, nf))
    src, fl = DeviceSource(traj, sel), FrameList(nf)
    for _ in range(5):
        run_pipeline(eng, src, fl, align="average")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps // 4):
        run_pipeline(eng, src, fl, align="average")
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / (reps // 4) * 1e3
    cap = CapturedPipeline(eng, src, fl, align="average")
    for _ in range(5):
        cap.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        cap.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / reps * 1e3
    digest = hashlib.sha1(cap.result.rmsf.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"C1 hipGraph replay: {graph:.4f} ms, eager {eager:.4f} ms per RMSF.py computation "
          f"({reps} replays, {os.path.relpath(_lib.LIB_PATH, ROOT)}; rmsf sha1 {digest})", flush=True)


if __name__ == "__main__":
    main()
