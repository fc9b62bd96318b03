#!/usr/bin/env python3
"""A/B in one process (round 5): ranges per chunk (S) of the flat balanced
plan when chunks outnumber workgroups (1M atoms: 2,930 chunks), at C4's
per-rank share (1M atoms x 2,500 frames): the whole launch + its fold-pack
against the two atom slabs of the N > 1 merge (each slab's launch + its
fold-pack), HIP-event medians, alternating.  Needs the temporary RMSF_SK_S
override (read per launch); results in profiles/r05_workloads/c4_share_s.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import _slab_bounds  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

eng = Engine()
n_atoms, nf = 1_000_000, int(sys.argv[1]) if len(sys.argv) > 1 else 2_500
traj = generate(eng, n_atoms, 0, nf, seed=0)
torch.cuda.synchronize()
ptr, fs, nc = traj.data_ptr(), traj.stride(0), 3 * n_atoms
shift = traj[0].reshape(-1).clone()
mean, m2 = eng.empty(nc), eng.empty(nc)
t_all = eng.empty(2 * nc)
S_VALUES = ["", "1", "2", "3", "4", "6"]
res = {}


def setS(v):
    if v:
        os.environ["RMSF_SK_S"] = v
    else:
        os.environ.pop("RMSF_SK_S", None)


for v in S_VALUES:
    setS(v)
    work = eng.empty(eng.balanced_workspace_bytes(n_atoms, nf) // 8 + 2)
    chunks = eng.balanced_slab_chunks(ptr, fs, nf, n_atoms)
    slabs = _slab_bounds(chunks, 2) if chunks >= 6 else None
    ts = [eng.empty(2 * (min(1024 * c1, nc) - 1024 * c0)) for c0, c1 in (slabs or [])]
    res[v] = dict(work=work, slabs=slabs, ts=ts, whole=[], two=[])

for rep in range(9):
    for v in S_VALUES:
        setS(v)
        r = res[v]
        for kind in ("whole", "two"):
            if kind == "two" and not r["slabs"]:
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            if kind == "whole":
                eng.accumulate_balanced(ptr, fs, nf, n_atoms, None, None, None, RMSF_MODE_WELFORD, r["work"])
                eng.fold_balanced_shift(r["work"], nc, 0, mean, m2, shift, None, t_all)
            else:
                for (c0, c1), t in zip(r["slabs"], r["ts"]):
                    eng.accumulate_balanced_slab(ptr, fs, nf, n_atoms, c0, c1, r["work"])
                    eng.fold_balanced_shift_slab(r["work"], nc, 0, mean, m2, shift, None, t, c0, c1)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                r[kind].append(e0.elapsed_time(e1))
floor = 12 * n_atoms * nf / 8e12 * 1e3
print(f"1M atoms x {nf} frames: accumulate + fold-pack, median of 8 (floor at 8 TB/s {floor:.3f} ms)")
for v in S_VALUES:
    r = res[v]
    w = float(np.median(r["whole"]))
    line = f"  S={v or 'default':7s} whole {w:.3f} ms ({floor / w:.3f})"
    if r["two"]:
        t = float(np.median(r["two"]))
        line += f"   2 slabs {t:.3f} ms ({floor / t:.3f}, {t / w:.3f}x whole)"
    print(line, flush=True)
