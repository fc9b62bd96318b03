#!/usr/bin/env python3
"""Is the torchrun rank step host-bound at the N = 8 share?  One process,
one GPU: run_pipeline over 100k atoms x 2,500 frames (C2's block at N = 8)
enqueued back to back; the host time per call (returning without a device
sync) against the device time per step (events around the whole run)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

eng = Engine()
for n_atoms, nf in ((100_000, 2_500), (100_000, 5_000), (100_000, 20_000)):
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    src = DeviceSource(traj, offset=0, n_traj=nf)
    fl = FrameList(nf)
    for _ in range(3):
        run_pipeline(eng, src, fl, block=(0, nf))
    torch.cuda.synchronize()
    k = 40
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = []
    a.record()
    t_all = time.perf_counter()
    for _ in range(k):
        t0 = time.perf_counter()
        run_pipeline(eng, src, fl, block=(0, nf))
        host.append(time.perf_counter() - t0)
    t_enq = time.perf_counter() - t_all
    b.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_all
    dev = a.elapsed_time(b) / k
    host.sort()
    print(f"{n_atoms} x {nf}: host per call median {host[k // 2] * 1e3:.3f} ms (p90 {host[int(k * 0.9)] * 1e3:.3f}), "
          f"enqueue of {k} {t_enq * 1e3:.1f} ms, device per step {dev:.3f} ms, wall per step {wall / k * 1e3:.3f} ms",
          flush=True)
    del traj, src
    torch.cuda.empty_cache()
