#!/usr/bin/env python3
"""A/B of rmsf_gather_frames -- the dense copy of a sparse selection's rows
(pipeline._Compactor) -- between the current library and an earlier build
(tools/_ab/librmsf_<v>.so, e.g. the round-5 one-float-per-thread kernel):
100k atoms x 20k frames, every 10th atom; HIP-event medians of alternating
rounds; copies compared bit for bit and against torch's own gather.
  python tools/ab_compact.py [VARIANT ...]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import LIB_PATH, SIGNATURES  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def lib(path):
    L = ctypes.CDLL(path)
    f = L.rmsf_gather_frames
    f.restype, f.argtypes = SIGNATURES["rmsf_gather_frames"]
    return L


eng = Engine()
n_atoms, nf = 100_000, 20_000
traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
libs = {"current": lib(LIB_PATH)}
for v in sys.argv[1:]:
    libs[v] = lib(os.path.join(ROOT, "tools", "_ab", f"librmsf_{v}.so"))
rows = torch.arange(nf, dtype=torch.int64, device="cuda")
for stride in (10, 220, 2):
    sel_h = np.arange(0, n_atoms, stride)
    sel = eng.sel_tensor(sel_h)
    n_sel = len(sel_h)
    outs = {k: torch.empty(nf, n_sel, 3, dtype=torch.float32, device="cuda") for k in libs}
    times = {k: [] for k in libs}
    for rnd in range(7):
        for k, L in libs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            rc = L.rmsf_gather_frames(traj.data_ptr(), 3 * n_atoms, rows.data_ptr(), nf, n_sel, sel.data_ptr(),
                                      outs[k].data_ptr(), eng.stream)
            b.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            if rnd:
                times[k].append(a.elapsed_time(b))
    want = traj[:, sel.long()]
    for k in libs:
        md = float(np.median(times[k]))
        print(f"1 in {stride:3d} ({n_sel} of {n_atoms}) {k:8s}: {md:.3f} ms; {12 * n_sel * nf / (md / 1e3) / 1e9:.0f} GB/s "
              f"selected written; equal to torch's gather: {bool(torch.equal(outs[k], want))}", flush=True)
    del outs, want
