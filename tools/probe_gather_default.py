#!/usr/bin/env python3
"""The default (frame-parallel) Welford over a gathered selection, timed
alone with HIP events: rmsf_accumulate_balanced (k_accum_atoms_sk, one atom
per lane) + the fold, at the selection sizes / densities of
tools/ab_seq_lib.py --shapes, beside the all-rows stream of the same
selected bytes.  Rates are algorithmic (12 B per selected atom-frame)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

eng = Engine()
for label, n_atoms, n_sel, nf in (("contiguous 100k", 100_000, 100_000, 20_000),
                                  ("gathered 100k of 120k", 120_000, 100_000, 20_000),
                                  ("third 100k of 300k", 300_000, 100_000, 4_000),
                                  ("sparse 100k of 1.5M", 1_500_000, 100_000, 800),
                                  ("sparse 20k of 300k", 300_000, 20_000, 5_000)):
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    sel = None if n_sel == n_atoms else eng.sel_tensor(np.sort(np.random.default_rng(1).choice(
        n_atoms, n_sel, replace=False)))
    work = eng.empty(eng.balanced_workspace_bytes(n_sel, nf) // 8 + 2)

    def acc():
        eng.accumulate_balanced(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sel, None, None, RMSF_MODE_WELFORD, work)

    acc()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        acc()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    md = float(np.median(ts))
    print(f"{label} x {nf}: accumulate {md:.3f} ms = {12 * n_sel * nf / (md / 1e3) / 1e9 / 8000:.3f} of 8 TB/s "
          f"(algorithmic)", flush=True)
    del traj, work
    torch.cuda.empty_cache()
