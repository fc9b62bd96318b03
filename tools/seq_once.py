#!/usr/bin/env python3
"""k_welford_seq alone at C2 (100k atoms x 20k frames, contiguous): 2 warm-up
launches and 3 timed ones (HIP events), for PMC passes (tools/pmc_seq.sh).
--gather: 100k of 120k atoms selected (k_welford_seq_atoms)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

import numpy as np  # noqa: E402

eng = Engine()
gather = "--gather" in sys.argv[1:]
n, nf = 100_000, 20_000
na = 120_000 if gather else n
traj = generate(eng, na, 0, nf, seed=0)
sel = eng.sel_tensor(np.sort(np.random.default_rng(1).choice(na, n, replace=False))) if gather else None
m, q = eng.empty(3 * n), eng.empty(3 * n)
work = eng.welford_sequential(traj.data_ptr(), 3 * na, nf, n, sel, 0, m, q)
eng.welford_sequential(traj.data_ptr(), 3 * na, nf, n, sel, 0, m, q, work)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    eng.welford_sequential(traj.data_ptr(), 3 * na, nf, n, sel, 0, m, q, work)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print("k_welford_seq" + ("_atoms" if gather else "") + " ms:", " ".join(f"{t:.3f}" for t in ts), flush=True)
