#!/usr/bin/env python3
"""The sequential Welford (rmsf_welford_sequential, RMSF.py:137-138 as
written) against the reference recurrence and against the balanced
accumulate + fold it would replace.

* exactness: mean and sumsquares bit for bit against the oracle's
  rank_sweep2 (RMSF.py:120-140 in numpy) on small cases, one batch and two
  batches continued at k0, and on 48 sampled atoms of the full 100k x 20k
  C2 trajectory;
* time: both forms at 100k atoms x 2,500 / 20,000 frames (HIP events,
  median), and the resulting RMSF against each other.

  python tools/seq_welford.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import rmsf_oracle as O  # noqa: E402
from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def bits_equal(a, b):
    return np.array_equal(np.asarray(a, np.float64).view(np.uint64), np.asarray(b, np.float64).view(np.uint64))


def times(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    eng = Engine()
    # exactness, small sizes (any atom count: one coordinate per lane)
    for n_atoms, nf in ((4096, 700), (1001, 333), (1002, 257), (5, 40)):
        traj = generate(eng, n_atoms, 0, nf, seed=5)
        host = traj.cpu().numpy()
        S = O.rank_sweep2(host, np.arange(n_atoms), None, 0, nf)
        nc = 3 * n_atoms
        m, q = eng.empty(nc), eng.empty(nc)
        eng.welford_sequential(traj.data_ptr(), nc, nf, n_atoms, None, 0, m, q)
        m2, q2 = eng.empty(nc), eng.empty(nc)
        cut = nf // 3
        eng.welford_sequential(traj.data_ptr(), nc, cut, n_atoms, None, 0, m2, q2)
        eng.welford_sequential(traj.data_ptr() + cut * nc * 4, nc, nf - cut, n_atoms, None, cut, m2, q2)
        torch.cuda.synchronize()
        one = bits_equal(m.cpu().numpy(), S[1].reshape(-1)) and bits_equal(q.cpu().numpy(), S[2].reshape(-1))
        two = bits_equal(m2.cpu().numpy(), S[1].reshape(-1)) and bits_equal(q2.cpu().numpy(), S[2].reshape(-1))
        print(f"{n_atoms:6d} atoms x {nf:5d} frames: one batch bit-exact {one}, two batches (k0 = {cut}) {two}",
              flush=True)
    # full C2 trajectory: time and 48 sampled atoms
    n_atoms, total = 100_000, 20_000
    traj = generate(eng, n_atoms, 0, total, seed=0)
    nc = 3 * n_atoms
    for nf in (2_500, 20_000):
        m, q = eng.empty(nc), eng.empty(nc)
        work = eng.welford_sequential(traj.data_ptr(), nc, nf, n_atoms, None, 0, m, q)
        seq = times(lambda: eng.welford_sequential(traj.data_ptr(), nc, nf, n_atoms, None, 0, m, q, work), 10)
        bw = eng.empty(eng.balanced_workspace_bytes(n_atoms, nf) // 8 + 2)
        bm, bq = eng.empty(nc), eng.empty(nc)

        def bal():
            eng.accumulate_balanced(traj.data_ptr(), nc, nf, n_atoms, None, None, None, RMSF_MODE_WELFORD, bw)
            eng.fold_balanced(bw, nc, RMSF_MODE_WELFORD, 0, bm, bq)

        b = times(bal, 10)
        r_seq, r_bal = eng.empty(n_atoms), eng.empty(n_atoms)
        eng.finalize(q, n_atoms, nf, r_seq)
        eng.finalize(bq, n_atoms, nf, r_bal)
        torch.cuda.synchronize()
        d = float((r_seq - r_bal).abs().max())
        gbs = 12.0 * n_atoms * nf / (seq * 1e-3) / 1e9
        print(f"100k x {nf:6d}: sequential {seq:.3f} ms ({gbs:.0f} GB/s, {gbs / 8000:.3f} of 8 TB/s), "
              f"balanced accumulate + fold {b:.3f} ms; max |RMSF seq - balanced| {d:.2e} A", flush=True)
        if nf == total:
            atoms = np.sort(np.random.default_rng(1).choice(n_atoms, 48, replace=False))
            cols = traj[:nf, atoms].cpu().numpy()
            S = O.rank_sweep2(cols, np.arange(48), None, 0, nf)
            got_m = m.view(n_atoms, 3)[atoms].cpu().numpy()
            got_q = q.view(n_atoms, 3)[atoms].cpu().numpy()
            print(f"  48 sampled atoms over {nf} frames bit-exact vs RMSF.py's recurrence: "
                  f"mean {bits_equal(got_m, S[1])}, sumsquares {bits_equal(got_q, S[2])}", flush=True)


if __name__ == "__main__":
    main()
