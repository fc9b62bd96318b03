#!/usr/bin/env python3
"""C5 (250k-atom XTC streamed from the host, GPU decode): frames/s of the
whole step against the decoder's batch size, slot count and read threads,
on one file written once (untimed).  The bench's c5_xtc mode uses the
defaults (batch ~2 GB of decoded frames, 3 slots, 16 threads).
  python tools/sweep_c5.py"""
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import run_pipeline  # noqa: E402
from rmsf_amd.sources import FrameList, XtcSource  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402
from rmsf_amd.xtc import write_xtc  # noqa: E402

eng = Engine()
n_atoms, nf = 250_000, 2048
d = tempfile.mkdtemp(prefix="rmsf_c5s_")
path = os.path.join(d, "c5.xtc")
try:
    for f in range(0, nf, 256):
        write_xtc(path, generate(eng, n_atoms, f, min(256, nf - f), seed=0).cpu().numpy(), append=f > 0)
    xb = os.path.getsize(path)
    ref = None
    for batch, slots, threads in ((None, 3, 16), (64, 3, 16), (128, 3, 16), (256, 3, 16), (128, 4, 16), (256, 4, 16),
                                  (128, 3, 24), (128, 2, 16), (None, 3, 16)):
        src = XtcSource(path, None, batch_frames=batch, n_slots=slots, n_threads=threads)
        fl = FrameList(nf)
        run_pipeline(eng, src, fl)
        torch.cuda.synchronize()
        ts = []
        for _ in range(4):
            t0 = time.perf_counter()
            res = run_pipeline(eng, src, fl)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        cs = float(res.rmsf.sum())
        ref = cs if ref is None else ref
        t = sorted(ts)[len(ts) // 2]
        print(f"batch {src.batch_frames:5d} slots {slots} threads {threads:2d}: {t * 1e3:7.2f} ms/step "
              f"{nf / t:8.0f} frames/s  {xb / t / 1e9:5.1f} GB/s of records  checksum equal {cs == ref}", flush=True)
        del src
finally:
    shutil.rmtree(d, ignore_errors=True)
