"""Sparse-selection aligned modes alone (round 6, verdict item 2): the
headline trajectory (100k atoms x 20k frames, aligned motion, HBM-resident)
with every 10th atom (CA-like) and every 220th (adk density) selected, frame-0
alignment and RMSF.py's two sweeps, compacted vs re-gathered.  HIP-event
spans per kernel family; run under rocprofv3 --kernel-trace --stats for the
per-kernel split.  python tools/probe_sparse.py [steps]
RMSF_AB_LIB=<path to a librmsf_hip.so build>: run with that build instead
(A/B on one box).  Stride 1 (contiguous C3) runs once, for the VEC4 path."""
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
from rmsf_amd.synth import generate, motion_table  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
if os.environ.get("RMSF_AB_LIB"):
    import rmsf_amd._lib as _L
    _L._lib = _L.load(os.environ["RMSF_AB_LIB"])
    print("library:", os.environ["RMSF_AB_LIB"], flush=True)
eng = Engine()
n_atoms, nf = 100_000, 20_000
traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
torch.cuda.synchronize()
fl = FrameList(nf)
CASES = ((1, "frame0"), (10, "frame0"), (10, "average"), (220, "average"), (220, "frame0"))
if os.environ.get("RMSF_PROBE_ONLY"):  # e.g. "10:frame0,10:average"
    CASES = tuple((int(c.split(":")[0]), c.split(":")[1]) for c in os.environ["RMSF_PROBE_ONLY"].split(","))
for stride, align in CASES:
    sel = np.arange(0, n_atoms, stride)
    src = DeviceSource(traj, sel)
    res = {}
    for compact in ((False,) if stride == 1 else (True, False)):
        for _ in range(2):
            run_pipeline(eng, src, fl, align=align, compact=compact)
        torch.cuda.synchronize()
        t = KernelTimer()
        t0 = time.perf_counter()
        for _ in range(steps):
            r = run_pipeline(eng, src, fl, align=align, compact=compact, timer=t)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps * 1e3
        res[compact] = r.rmsf
        _, s_ms, _ = t.totals("superpose")
        _, a_ms, _ = t.totals("accumulate")
        sweeps = 2 if align == "average" else 1
        gbs = 12 * len(sel) * nf * sweeps / (dt / 1e3) / 1e9
        print(f"1 in {stride:3d} ({len(sel)} of {n_atoms}) {align:7s} compact={compact!s:5s}: {dt:7.3f} ms/step "
              f"(superpose {s_ms / steps:6.3f}, accumulate {a_ms / steps:6.3f}; selected {gbs:6.0f} GB/s = "
              f"{gbs / 8000:.3f} of 8 TB/s)", flush=True)
    if stride > 1:
        print(f"   same bits: {bool(torch.equal(res[True], res[False]))}", flush=True)
    del src
