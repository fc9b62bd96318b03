"""Batch-size probe of the aligned path (C3 / RMSF.py's two sweeps) on the
headline trajectory (100k atoms x 20k frames, HBM-resident): with batches
that fit the 256 MB memory-side cache, the accumulate's second read of a
batch could come from that cache instead of HBM.  HIP-event spans per
kernel family.  python tools/probe_batch.py [steps] [align]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import KernelTimer, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
align = sys.argv[2] if len(sys.argv) > 2 else "frame0"
eng = Engine()
n_atoms, nf = 100_000, 20_000
traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
torch.cuda.synchronize()
fl = FrameList(nf)
src = DeviceSource(traj, None)
base = None
for mb in (nf, 4096, 1024, 512, 256, 128, 64):
    for _ in range(2):
        run_pipeline(eng, src, fl, align=align, max_batch=mb)
    torch.cuda.synchronize()
    t = KernelTimer()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = run_pipeline(eng, src, fl, align=align, max_batch=mb, timer=t)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    _, s_ms, _ = t.totals("superpose")
    _, a_ms, _ = t.totals("accumulate")
    if base is None:
        base = r.rmsf
    d = float((r.rmsf - base).abs().max())
    print(f"{align} batch {mb:5d} frames ({12 * n_atoms * mb / 2**20:7.1f} MiB): {dt:7.3f} ms/step "
          f"(superpose {s_ms / steps:6.3f}, accumulate {a_ms / steps:6.3f}); max |d rmsf| vs whole {d:.2e}", flush=True)
