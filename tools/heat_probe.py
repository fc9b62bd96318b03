#!/usr/bin/env python3
"""Does the headline stream slow down under sustained load?  One process:
the C2 Welford step (k_welford_flat_sk + fold, 100k atoms x 20k frames)
launched back to back for --seconds, each launch timed by HIP events; the
medians per 10-second window are printed as they come, with the effective
rate (fraction of 8 TB/s).  --exact interleaves k_welford_seq launches.
  python tools/heat_probe.py [--seconds 90] [--exact]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90)
    ap.add_argument("--exact", action="store_true")
    a = ap.parse_args()
    eng = Engine()
    n, nf = 100_000, 20_000
    traj = generate(eng, n, 0, nf, seed=0)
    work = eng.empty(eng.balanced_workspace_bytes(n, nf) // 8 + 2)
    m, q = eng.empty(3 * n), eng.empty(3 * n)
    sw = eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q) if a.exact else None
    gb = 12 * n * nf / 1e9

    def launch():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.accumulate_balanced(traj.data_ptr(), 3 * n, nf, n, None, None, None, RMSF_MODE_WELFORD, work)
        e1.record()
        x = None
        if a.exact:
            x = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            x[0].record()
            eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q, sw)
            x[1].record()
        return (e0, e1), x

    t_end = time.perf_counter() + a.seconds
    t_win = time.perf_counter() + 10
    win, win_x, k = [], [], 0
    t_start = time.perf_counter()
    while time.perf_counter() < t_end:
        evs = [launch() for _ in range(8)]
        torch.cuda.synchronize()
        win += [e0.elapsed_time(e1) for (e0, e1), _ in evs]
        win_x += [x[0].elapsed_time(x[1]) for _, x in evs if x is not None]
        k += len(evs)
        if time.perf_counter() >= t_win:
            md = float(np.median(win))
            line = (f"t={time.perf_counter() - t_start:5.1f}s launches {k:5d}  flat median {md:.3f} ms "
                    f"({gb / md / 8:.3f} of 8 TB/s) min {min(win):.3f} max {max(win):.3f}")
            if win_x:
                mx = float(np.median(win_x))
                line += f"  | seq median {mx:.3f} ms ({gb / mx / 8:.3f})"
            print(line, flush=True)
            win, win_x = [], []
            t_win += 10


if __name__ == "__main__":
    main()
