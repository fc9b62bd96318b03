#!/usr/bin/env python3
"""Workgroup-count sweep of the balanced accumulate kernels (not product code).

For each kernel variant -- float4 Welford (C2), aligned Welford and aligned
sum (C3 / RMSF.py sweeps), gathered unaligned Welford -- times
rmsf_accumulate_balanced at several workgroup counts against the split grid
(rmsf_accumulate, auto splits), HIP events on the launch stream, 100k atoms x
20k frames resident in HBM.

  python tools/tune_groups.py [--frames 20000] [--atoms 100000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--atoms", type=int, default=100_000)
    ap.add_argument("--frames", type=int, default=20_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1, help="repeat the whole sweep (run-to-run spread)")
    ap.add_argument("--splits", default="", help="extra split counts for the split grid")
    ap.add_argument("--groups", default="256,512,768,1024,1536,2048,3072,4096,6144,8192")
    a = ap.parse_args()
    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_MODE_WELFORD
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table

    eng = Engine()
    n, nf = a.atoms, a.frames
    traj = generate(eng, n, 0, nf, seed=0, motion=motion_table(1, nf))
    ref, info = eng.reference_setup(n, frame_ptr=traj.data_ptr())
    xf = eng.empty(nf, 16)
    wk = eng.empty(eng.workspace_bytes(n, nf) // 8 + 1)
    eng.superpose(traj.data_ptr(), 3 * n, nf, n, None, None, ref, info, xf, wk)
    sel = torch.arange(0, n, 2, dtype=torch.int32, device=eng.device)
    # C2's own data (no rigid motion: the bench's input) next to the C3 data
    traj_c2 = generate(eng, n, 0, nf, seed=0) if os.environ.get("TUNE_C2DATA", "1") == "1" else traj
    torch.cuda.synchronize()
    del wk
    groups = [int(g) for g in a.groups.split(",")]
    work = eng.empty(max(eng.balanced_workspace_bytes(n, nf, g) for g in groups + [0]) // 8 + 2)
    s_max = max([eng.splits(n, nf, True), eng.splits(n, nf, False)] + [int(x) for x in a.splits.split(",") if x])
    p0, p1 = eng.empty(s_max, 3 * n), eng.empty(s_max, 3 * n)
    mb = 12 * n * nf

    def timeit(fn):
        s = torch.cuda.current_stream()
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record(s)
            fn()
            e1.record(s)
        torch.cuda.synchronize()
        return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))

    variants = {
        "flat_welford": dict(sel=None, xf=None, info=None, mode=RMSF_MODE_WELFORD, aligned=False, n_sel=n),
        "flat_welford_c2data": dict(sel=None, xf=None, info=None, mode=RMSF_MODE_WELFORD, aligned=False, n_sel=n,
                                    traj=traj_c2),
        "aligned_welford": dict(sel=None, xf=xf, info=info, mode=RMSF_MODE_WELFORD, aligned=True, n_sel=n),
        "aligned_sum": dict(sel=None, xf=xf, info=info, mode=RMSF_MODE_SUM, aligned=True, n_sel=n),
        "gather_welford": dict(sel=sel, xf=None, info=None, mode=RMSF_MODE_WELFORD, aligned=False, n_sel=n // 2),
    }
    only = os.environ.get("TUNE_ONLY")
    if only:
        variants = {k: v for k, v in variants.items() if k in only.split(",")}
    out = {}
    for name, v in [(k, v) for _ in range(a.rounds) for k, v in variants.items()]:
        ns = v["n_sel"]
        x = v.get("traj", traj)
        bytes_ = 12 * ns * nf
        s = eng.splits(ns, nf, v["aligned"])
        t = timeit(lambda: eng.accumulate(x.data_ptr(), 3 * n, nf, ns, v["sel"], v["xf"], v["info"], v["mode"], s,
                                          p0, p1 if v["mode"] == RMSF_MODE_WELFORD else None))
        row = {"split_grid": {"splits": s, "ms": t, "frac": bytes_ / t / 1e9 / 8000}}
        for s2 in [int(x) for x in a.splits.split(",") if x]:
            t = timeit(lambda: eng.accumulate(x.data_ptr(), 3 * n, nf, ns, v["sel"], v["xf"], v["info"], v["mode"],
                                              s2, p0, p1 if v["mode"] == RMSF_MODE_WELFORD else None))
            row[f"S{s2}"] = {"ms": t, "frac": bytes_ / t / 1e9 / 8000}
        for g in groups:
            t = timeit(lambda: eng.accumulate_balanced(x.data_ptr(), 3 * n, nf, ns, v["sel"], v["xf"], v["info"],
                                                       v["mode"], work, g))
            row[f"G{g}"] = {"ms": t, "frac": bytes_ / t / 1e9 / 8000}
        out[name] = row
        best = min((k for k in row if k.startswith("G")), key=lambda k: row[k]["ms"])
        print(f"{name:16s} split({s}) {row['split_grid']['ms']:.3f} ms  best {best} {row[best]['ms']:.3f} ms  "
              + " ".join(f"{k}:{row[k]['ms']:.3f}" for k in row if k[0] in "GS"), flush=True)
    del mb
    print(json.dumps({"atoms": n, "frames": nf, "results": out}))


if __name__ == "__main__":
    main()
