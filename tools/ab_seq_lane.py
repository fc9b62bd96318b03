#!/usr/bin/env python3
"""A/B in one process: the sequential Welford
(RMSF.py:137-138 as written, k_welford_seq) with its per-frame coefficients
from the k_seq_coef table (scalar loads, "table") against coefficients
computed per 64-frame window by the wave itself and broadcast by v_readlane
("lane").  Alternating, HIP-event medians, bits compared; needs the temporary
RMSF_SEQ_COEF switch (read per call).  100k atoms x 20k frames, plus a
gathered selection and a ragged batch for the bit check.  Result in
profiles/r05_workloads/seq_welford_lane.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def set_variant(name):
    if name == "lane":
        os.environ["RMSF_SEQ_COEF"] = "lane"
    else:
        os.environ.pop("RMSF_SEQ_COEF", None)


eng = Engine()
n, nf = 100_000, 20_000
traj = generate(eng, n, 0, nf, seed=0)
m, q = eng.empty(3 * n), eng.empty(3 * n)
work = eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q)
res = {"table": [], "lane": []}
outs = {}
for rep in range(7):
    for name in ("table", "lane"):
        set_variant(name)
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q, work)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf, n, None, 0, m, q, work)
        b.record()
        torch.cuda.synchronize()
        res[name].append(a.elapsed_time(b))
        outs[name] = (m.cpu().numpy().copy(), q.cpu().numpy().copy())
same = all(np.array_equal(outs["table"][i].view(np.uint64), outs["lane"][i].view(np.uint64)) for i in (0, 1))
print(f"100k atoms x 20k frames, k_welford_seq<8>, one process, alternating, {len(res['table'])} rounds")
for k, v in res.items():
    med = float(np.median(v))
    print(f"  {k:5s} " + " ".join(f"{x:.3f}" for x in v) + f"  median {med:.3f} ms  {24e9 / (med / 1e3) / 8e12:.3f} of 8 TB/s")
print("  bitwise equal (mean, sumsquares):", same)
# more shapes for the bits: gathered selection, ragged batches continued at k0 > 0, windows not aligned to 64
sel = np.sort(np.random.default_rng(1).choice(n, 777, replace=False))
sdev = eng.sel_tensor(sel)
ok = True
for nf2, k0 in ((1, 0), (7, 0), (63, 5), (64, 64), (129, 1000), (1000, 3)):
    got = []
    for name in ("table", "lane"):
        set_variant(name)
        mm = torch.tensor(np.full(3 * len(sel), 50.0), device=eng.device)
        qq = torch.tensor(np.full(3 * len(sel), 1.0), device=eng.device)
        eng.welford_sequential(traj.data_ptr(), 3 * n, nf2, len(sel), sdev, k0, mm, qq)
        torch.cuda.synchronize()
        got.append((mm.cpu().numpy(), qq.cpu().numpy()))
    e = all(np.array_equal(got[0][i].view(np.uint64), got[1][i].view(np.uint64)) for i in (0, 1))
    ok &= e
    print(f"  gathered 777 atoms, {nf2} frames from k0={k0}: bitwise equal {e}")
print("ALL_EQUAL", same and ok)
