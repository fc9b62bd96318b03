"""One sparse-selection aligned configuration for rocprofv3 --pmc passes
(round 6, verdict item 2): 100k atoms x 20k frames (aligned motion, HBM),
every STRIDE-th atom selected, ALIGN in {frame0, average}, compact 1/0,
STEPS pipeline runs after one warm-up.
  python tools/sparse_once.py STRIDE ALIGN COMPACT [STEPS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402

stride, align, compact = int(sys.argv[1]), sys.argv[2], bool(int(sys.argv[3]))
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
eng = Engine()
n_atoms, nf = 100_000, 20_000
traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
src = DeviceSource(traj, np.arange(0, n_atoms, stride))
for _ in range(1 + steps):
    r = run_pipeline(eng, src, FrameList(nf), align=align, compact=compact)
torch.cuda.synchronize()
print(f"every {stride}th atom, {align}, compact={compact}: rmsf[0] = {float(r.rmsf[0]):.6f}")
