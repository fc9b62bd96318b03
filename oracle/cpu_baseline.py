"""bench.py's ``cpu_baseline`` leg -- BENCH/TEST INFRASTRUCTURE ONLY.

Times the oracle's numpy restatement of RMSF.py's per-rank loop on the host
cores, the way ``mpirun -n P python RMSF.py`` would run it: P independent
processes, one BLAS/OMP thread each (RMSF.py:23-25), each owning one
contiguous frame block (RMSF.py:65-69) of the same synthetic workload, then
the Chan fold of the P partials (RMSF.py:143).  Frames are generated before
the timed loop (RMSF.py re-decodes an XTC instead, so this baseline is
optimistic: no decode and no per-frame re-selection).

Run as ``python -m oracle.cpu_baseline --worker ...`` (one process per
core, started with subprocess -- never fork()ed from a GPU process).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

_ENV1 = {"MKL_NUM_THREADS": "1", "NUMEXPR_NUM_THREADS": "1", "OMP_NUM_THREADS": "1", "OPENBLAS_NUM_THREADS": "1"}


def _worker(a):
    os.environ.update(_ENV1)
    import numpy as np

    from oracle import rmsf_oracle as O
    from oracle import synth as SY

    motion = None
    if a.align != "none":
        motion = np.load(a.motion)
    traj = SY.frames(a.seed, a.n_atoms, a.f0, a.nf, motion)
    sel = np.arange(a.n_atoms)
    t0 = time.perf_counter()
    if a.align == "none":
        S = O.rank_sweep2(traj, sel, None, 0, a.nf)
    else:
        ref0 = SY.frames(a.seed, a.n_atoms, 0, 1, motion)[0]
        ref_com, ref_c = O.centred_reference(ref0[sel])
        S = O.rank_sweep2(traj, sel, None, 0, a.nf, ref_c, ref_com)
    dt = time.perf_counter() - t0
    np.savez(a.out, n=S[0], mean=S[1], m2=S[2], dt=dt)


def run(n_atoms: int, frames_per_proc: int, procs: int | None = None, seed: int = 0, align: str = "none",
        motion=None) -> dict:
    """Launch ``procs`` worker processes; returns the atom-frames/s figure."""
    import numpy as np

    from oracle import rmsf_oracle as O

    if procs is None:
        procs = max(1, min(len(os.sched_getaffinity(0)), 16))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **_ENV1)
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    with tempfile.TemporaryDirectory(prefix="rmsf_cpu_") as tmp:
        mpath = os.path.join(tmp, "motion.npy")
        if motion is not None:
            np.save(mpath, motion)
        ps, outs = [], []
        for r in range(procs):
            out = os.path.join(tmp, f"part{r}.npz")
            outs.append(out)
            cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--worker", "--n-atoms", str(n_atoms), "--f0",
                   str(r * frames_per_proc), "--nf", str(frames_per_proc), "--seed", str(seed), "--align", align,
                   "--motion", mpath, "--out", out]
            ps.append(subprocess.Popen(cmd, env=env, cwd=root))
        for p in ps:
            if p.wait() != 0:
                raise RuntimeError("cpu baseline worker failed")
        parts, dts = [], []
        for out in outs:
            d = np.load(out)
            parts.append([int(d["n"]), d["mean"], d["m2"]])
            dts.append(float(d["dt"]))
        t0 = time.perf_counter()
        Data = O.chan_fold(parts)  # RMSF.py:143 (root fold)
        np.sqrt(Data[2].sum(axis=1) / Data[0])  # RMSF.py:146
        t_merge = time.perf_counter() - t0
    total = n_atoms * frames_per_proc * procs
    wall = max(dts) + t_merge
    return {"value": total / wall, "unit": "atom-frames/s", "cores": procs, "kind": "port",
            "sample": f"{n_atoms} atoms x {frames_per_proc * procs} frames ({frames_per_proc}/process), "
                      f"align={align}, numpy restatement of RMSF.py per-rank loop, {procs} processes x 1 thread, "
                      f"frames pre-generated (no XTC decode): optimistic",
            "seconds": wall, "cpu_seconds": sum(dts)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--n-atoms", type=int, default=100_000)
    ap.add_argument("--f0", type=int, default=0)
    ap.add_argument("--nf", type=int, default=16)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--align", default="none")
    ap.add_argument("--motion", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--procs", type=int, default=None)
    a = ap.parse_args()
    if a.worker:
        _worker(a)
    else:
        print(json.dumps(run(a.n_atoms, a.nf, a.procs, a.seed, a.align)))
