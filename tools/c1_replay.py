#!/usr/bin/env python3
"""C1 shape (3341 atoms, 214 selected, 98 frames, RMSF.py's two sweeps) as a
captured pipeline replayed N times -- for a kernel trace of one replay's
launches.  python tools/c1_replay.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import CapturedPipeline, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
eng = Engine()
n_atoms, nf = 3341, 98
sel = np.sort(np.random.default_rng(12).choice(n_atoms, 214, replace=False))
traj = generate(eng, n_atoms, 0, nf, seed=11, motion=motion_table(13, nf))
src = DeviceSource(traj, sel)
fl = FrameList(nf)
cap = CapturedPipeline(eng, src, fl, align="average")
for _ in range(3):
    cap.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    cap.replay()
torch.cuda.synchronize()
print(f"replay {1e3 * (time.perf_counter() - t0) / reps:.4f} ms")
t0 = time.perf_counter()
for _ in range(reps):
    run_pipeline(eng, src, fl, align="average")
torch.cuda.synchronize()
print(f"eager {1e3 * (time.perf_counter() - t0) / reps:.4f} ms")
