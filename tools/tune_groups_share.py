#!/usr/bin/env python3
"""Workgroup count of the flat balanced Welford grid at the strong-scaling
shares: accumulate + fold device time for n_groups in a range, at 100k atoms
x {2,500, 5,000, 20,000} frames (0 = the library's default, 3 per CU).

  python tools/tune_groups_share.py [--reps 15]
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
from rmsf_amd.synth import generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    eng = Engine(torch.device("cuda", 0))
    n = 100_000
    traj = generate(eng, n, 0, 20_000, seed=0)
    torch.cuda.synchronize()
    mean, m2 = eng.empty(3 * n), eng.empty(3 * n)
    for nf in (2_500, 5_000, 20_000):
        row = {"frames": nf}
        for g in (0, 256, 384, 512, 640, 0, 512):
            work = eng.empty(eng.balanced_workspace_bytes(n, nf, g) // 8 + 2)

            def once():
                eng.accumulate_balanced(traj.data_ptr(), 3 * n, nf, n, None, None, None, RMSF_MODE_WELFORD, work, g)
                eng.fold_balanced(work, 3 * n, RMSF_MODE_WELFORD, 0, mean, m2)
            for _ in range(3):
                once()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    once()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 5)
            ts.sort()
            row[f"G{g}_ms"] = round(ts[len(ts) // 2], 4)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
