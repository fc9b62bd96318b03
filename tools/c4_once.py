"""C4's per-rank share against the headline shape with the same bytes (round
6, verdict item 4): the unaligned flat Welford stream (rmsf_accumulate_balanced,
k_welford_flat_sk) over 1M atoms x 2,500 frames and over 100k atoms x 25,000
frames (2.5e9 atom-frames = 30 GB each), 5 launches each, HIP-event medians.
Run alone, or under rocprofv3 --pmc for the per-launch counters.
  python tools/c4_once.py [launches]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 5
eng = Engine()
for n_atoms, nf in ((1_000_000, 2_500), (100_000, 25_000)):
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    work = eng.empty(eng.balanced_workspace_bytes(n_atoms, nf) // 8 + 2)
    acc0, acc1 = eng.empty(3 * n_atoms), eng.empty(3 * n_atoms)
    ts = []
    for i in range(k + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.accumulate_balanced(traj.data_ptr(), 3 * n_atoms, nf, n_atoms, None, None, None, RMSF_MODE_WELFORD, work)
        b.record()
        eng.fold_balanced(work, 3 * n_atoms, RMSF_MODE_WELFORD, 0, acc0, acc1)
        torch.cuda.synchronize()
        if i:
            ts.append(a.elapsed_time(b))
    md = float(np.median(ts))
    print(f"{n_atoms} atoms x {nf} frames: accumulate {md:.3f} ms = {12 * n_atoms * nf / (md / 1e3) / 1e12:.3f} TB/s "
          f"= {12 * n_atoms * nf / (md / 1e3) / 8e12:.3f} of 8 TB/s", flush=True)
    del traj, work
    torch.cuda.empty_cache()
