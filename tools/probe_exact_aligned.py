"""Cost of the exact aligned path (rmsf_superpose_sequential /
rmsf_accumulate_sequential, the auto default below 256 frames) against the
frame-parallel one, by shape: HIP-event spans per kernel family.
  python tools/probe_exact_aligned.py [steps]"""
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

if os.environ.get("RMSF_AB_LIB"):
    import rmsf_amd._lib as _L
    _L._lib = _L.load(os.environ["RMSF_AB_LIB"])
    print("library:", os.environ["RMSF_AB_LIB"], flush=True)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
eng = Engine()
SHAPES = ((47_681, 214, 10), (100_000, 100_000, 100), (100_000, 10_000, 200), (1_000_000, 1_000_000, 32))
if os.environ.get("PROBE_SHAPE"):  # e.g. "1": only SHAPES[1]
    SHAPES = tuple(SHAPES[int(i)] for i in os.environ["PROBE_SHAPE"].split(","))
for n_atoms, n_sel, nf in SHAPES:
    traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    sel = None if n_sel == n_atoms else np.linspace(0, n_atoms - 1, n_sel).astype(np.int64)
    src = DeviceSource(traj, sel)
    fl = FrameList(nf)
    for align in ("frame0", "average"):
        res = {}
        for exact in (False, True):
            run_pipeline(eng, src, fl, align=align, exact=exact)
            torch.cuda.synchronize()
            t = KernelTimer()
            t0 = time.perf_counter()
            for _ in range(steps):
                r = run_pipeline(eng, src, fl, align=align, exact=exact, timer=t)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps * 1e3
            res[exact] = r.rmsf
            fam = {k: t.totals(k)[1] / steps for k in list(t.spans)}
            spans = ", ".join(f"{k} {v:.3f}" for k, v in sorted(fam.items()))
            print(f"{n_sel:>9,} of {n_atoms:>9,} x {nf:4d} {align:7s} exact={exact!s:5s}: {dt:9.3f} ms/run  [{spans}]",
                  flush=True)
        print(f"   max |d rmsf| {float((res[True] - res[False]).abs().max()):.2e}", flush=True)
    del traj, src
    torch.cuda.empty_cache()
