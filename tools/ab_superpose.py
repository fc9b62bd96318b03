#!/usr/bin/env python3
"""A/B of rmsf_superpose between two builds of the library in one process
(tools/_ab/librmsf_old.so vs the current one): transform records compared
byte for byte, then timed.  python tools/ab_superpose.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import LIB_PATH  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402

P = ctypes.c_void_p
libs = {"old": ctypes.CDLL(os.path.join(ROOT, "tools", "_ab", "librmsf_old.so")), "new": ctypes.CDLL(LIB_PATH)}
for L in libs.values():
    L.rmsf_superpose.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, P, P, P, P, P, ctypes.c_size_t, P]
    L.rmsf_superpose_workspace_bytes.restype = ctypes.c_size_t
    L.rmsf_superpose_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int64]
eng = Engine()
for n_sel, nf, gather, masses in ((100_000, 20_000, False, False), (100_000, 2_500, False, False),
                                  (214, 98, True, False), (3000, 777, True, True), (5, 65, False, True)):
    n_atoms = n_sel + 7 if gather else n_sel
    traj = generate(eng, n_atoms, 0, nf, seed=3, motion=motion_table(4, nf))
    sel = torch.tensor(np.sort(np.random.default_rng(1).choice(n_atoms, n_sel, replace=False)).astype(np.int32),
                       device=eng.device) if gather else None
    m = torch.tensor(np.random.default_rng(2).uniform(1, 16, n_sel), device=eng.device) if masses else None
    ref, info = eng.reference_setup(n_sel, frame_ptr=traj.data_ptr(), sel=sel, masses=m)
    wb = libs["new"].rmsf_superpose_workspace_bytes(n_sel, nf)
    work = torch.empty(max(wb, 16) // 8 + 2, dtype=torch.float64, device=eng.device)
    out, ms = {}, {}
    for k, L in libs.items():
        xf = torch.full((nf, 16), float("nan"), dtype=torch.float64, device=eng.device)

        def run():
            rc = L.rmsf_superpose(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sel.data_ptr() if gather else None,
                                  m.data_ptr() if masses else None, ref.data_ptr(), info.data_ptr(), xf.data_ptr(),
                                  work.data_ptr(), work.numel() * 8, eng.stream)
            assert rc == 0, rc
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[k], ms[k] = xf.cpu().numpy(), sorted(ts)[len(ts) // 2]
    same = np.array_equal(out["old"].view(np.uint64), out["new"].view(np.uint64))
    print(f"n_sel {n_sel:6d} frames {nf:5d} gather {gather} masses {masses}: bitwise equal {same}; "
          f"superpose old {ms['old']:.4f} ms new {ms['new']:.4f} ms", flush=True)
