#!/usr/bin/env python3
"""A/B in one process (round 5): the sequential Welford (RMSF.py:137-138 as
written) in the kept two-block form against a ring of NB blocks of U frames
(k_welford_seq_ring: NB - 1 blocks of loads in flight while one folds, the
coefficients double-buffered).  Needs the temporary RMSF_SEQ_RING switch
(<U><NB>, read per call).  Alternating rounds, HIP-event medians at 100k x
20k (contiguous) and 100k-of-120k atoms (gathered), bits compared."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

ENV = os.environ.get("AB_SWITCH", "RMSF_SEQ_RING")  # RMSF_SEQ_BUF: the buffer-load ring (both switches since removed)
VARIANTS = sys.argv[1:] or ["kept", "82", "84", "86", "44", "48", "64"]


def setv(v):
    if v == "kept":
        os.environ.pop(ENV, None)
    else:
        os.environ[ENV] = v


eng = Engine()
nf = 20_000
CASES = (("contiguous 100k", 100_000, 100_000), ("gathered 100k of 120k", 120_000, 100_000))
if os.environ.get("AB_CONTIGUOUS_ONLY"):
    CASES = CASES[:1]
for label, n_atoms, n_sel in CASES:
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    sel = None if n_sel == n_atoms else eng.sel_tensor(np.sort(np.random.default_rng(1).choice(n_atoms, n_sel,
                                                                                              replace=False)))
    m, q = eng.empty(3 * n_sel), eng.empty(3 * n_sel)
    work = eng.welford_sequential(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sel, 0, m, q)
    res = {v: [] for v in VARIANTS}
    outs = {}
    for rep in range(5):
        for v in VARIANTS:
            setv(v)
            eng.welford_sequential(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sel, 0, m, q, work)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            eng.welford_sequential(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sel, 0, m, q, work)
            b.record()
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b))
            outs[v] = (m.cpu().numpy().copy(), q.cpu().numpy().copy())
    print(f"{label} x {nf} frames, alternating, 5 rounds:", flush=True)
    for v in VARIANTS:
        med = float(np.median(res[v]))
        same = all(np.array_equal(outs[v][i].view(np.uint64), outs["kept"][i].view(np.uint64)) for i in (0, 1))
        print(f"  {v:5s} median {med:.3f} ms  {12 * n_sel * nf / (med / 1e3) / 8e12:.3f} of 8 TB/s  "
              f"[{' '.join(f'{x:.3f}' for x in res[v])}]  bits == kept: {same}", flush=True)
    del traj
    torch.cuda.empty_cache()
# ragged shapes for the bits
traj = generate(eng, 5000, 0, 700, seed=3)
ok = True
for nf2, k0 in ((1, 0), (7, 0), (31, 5), (33, 64), (129, 1000), (700, 3)):
    base = None
    for v in VARIANTS:
        setv(v)
        mm = torch.tensor(np.full(3 * 5000, 50.0), device=eng.device)
        qq = torch.tensor(np.full(3 * 5000, 1.0), device=eng.device)
        eng.welford_sequential(traj.data_ptr(), 3 * 5000, nf2, 5000, None, k0, mm, qq)
        torch.cuda.synchronize()
        got = (mm.cpu().numpy().view(np.uint64), qq.cpu().numpy().view(np.uint64))
        if base is None:
            base = got
        ok &= all(np.array_equal(got[i], base[i]) for i in (0, 1))
print("ragged shapes all equal:", ok)
