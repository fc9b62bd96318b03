#!/usr/bin/env python3
"""A/B in one process, kept as the record of a measurement: the sequential
Welford with and without the per-block special-value check.  It needs the
removed RMSF_SEQ_HOIST switch (read per call); the result is in
profiles/r04_workloads/seq_welford_variants.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402

eng = Engine()
n, nf = 100_000, 20_000
traj = generate(eng, n, 0, nf, seed=0)
m, q = eng.empty(3 * n), eng.empty(3 * n)
work = eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q)
res = {"kept": [], "hoist": []}
outs = {}
for rep in range(6):
    for name in ("kept", "hoist"):
        if name == "hoist":
            os.environ["RMSF_SEQ_HOIST"] = "1"
        else:
            os.environ.pop("RMSF_SEQ_HOIST", None)
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q, work)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q, work)
        b.record()
        torch.cuda.synchronize()
        res[name].append(a.elapsed_time(b))
        outs[name] = (m.cpu().numpy().copy(), q.cpu().numpy().copy())
same = all(np.array_equal(outs["kept"][i].view(np.uint64), outs["hoist"][i].view(np.uint64)) for i in (0, 1))
for k, v in res.items():
    print(k, " ".join(f"{x:.3f}" for x in v), "median", f"{np.median(v):.3f} ms")
print("bitwise equal", same)
