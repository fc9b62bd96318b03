#!/usr/bin/env python3
"""Why does k_welford_seq time 4.66 ms inside bench.py's c2_exact mode but
4.1-4.2 ms in the one-kernel A/B scripts (same 100k x 20k frames)?  One
process, HIP events per launch, in this order:
  A  the kernel alone, 5 launches (as tools/ab_seq_ring.py)
  B  the pipeline's exact run (run_pipeline(exact=True)), 5 steps
  C  20 headline steps (k_welford_flat_sk stream), then A again
  D  the kernel alone with a fresh coefficient workspace and zeroed state
     per launch (what the pipeline does per step)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import KernelTimer, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

eng = Engine()
n, nf = 100_000, 20_000
traj = generate(eng, n, 0, nf, seed=0)
torch.cuda.synchronize()
m, q = eng.empty(3 * n), eng.empty(3 * n)


def direct(reps, fresh=False):
    work = eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q)
    out = []
    for _ in range(reps):
        if fresh:
            mm, qq = eng.zeros(3 * n), eng.zeros(3 * n)
            w = None
        else:
            mm, qq, w = m, q, work
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, mm, qq, w)
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return out


def fmt(t):
    return f"median {np.median(t):.3f} ms [{' '.join(f'{x:.3f}' for x in t)}]"


print("A direct:", fmt(direct(5)), flush=True)
src = DeviceSource(traj, offset=0, n_traj=nf)
fl = FrameList(nf)
run_pipeline(eng, src, fl, block=(0, nf), exact=True)
torch.cuda.synchronize()
xt = KernelTimer()
for _ in range(5):
    run_pipeline(eng, src, fl, block=(0, nf), exact=True, timer=xt)
torch.cuda.synchronize()
print("B pipeline exact:", fmt(xt.ms("accumulate")), flush=True)
ht = KernelTimer()
t0 = time.perf_counter()
for _ in range(20):
    run_pipeline(eng, src, fl, block=(0, nf), timer=ht)
torch.cuda.synchronize()
print(f"C headline 20 steps: accumulate {fmt(ht.ms('accumulate')[-5:])} (last 5), "
      f"{(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step", flush=True)
print("C then direct:", fmt(direct(5)), flush=True)
print("D direct, fresh state per launch:", fmt(direct(5, fresh=True)), flush=True)
xt = KernelTimer()
for _ in range(5):
    run_pipeline(eng, src, fl, block=(0, nf), exact=True, timer=xt)
torch.cuda.synchronize()
print("B again:", fmt(xt.ms("accumulate")), flush=True)
