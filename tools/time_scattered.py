"""Times RMSF.run(frames=<random 50 % mask>) over an HBM-resident trajectory
(100k atoms x 2,000 frames; runs average 2 frames) with the gathered-batch
path (sources.SCATTER_RUN = 8, the default) and with one batch per run
(SCATTER_RUN = 0), for align None / frame0.  Not product code."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd import RMSF, sources  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402

eng = Engine()
n_atoms, nf = 100_000, 2000
traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
mask = np.random.default_rng(0).random(nf) < 0.5
mask[0] = True
for align in (None, "frame0"):
    res = {}
    for run_len in (8, 0):
        sources.SCATTER_RUN = run_len
        RMSF(traj, align=align).run(frames=mask)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            r = RMSF(traj, align=align).run(frames=mask).results.rmsf
        torch.cuda.synchronize()
        res[run_len] = ((time.perf_counter() - t0) / 3 * 1e3, r)
    d = float(np.abs(res[8][1] - res[0][1]).max())
    print(f"align={align}: {mask.sum()} scattered frames of {nf}: gathered batches {res[8][0]:.1f} ms, "
          f"one batch per run {res[0][0]:.1f} ms, max |dRMSF| {d:.2e} A")
