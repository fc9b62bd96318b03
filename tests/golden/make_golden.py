"""Regenerate the golden fixtures in tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).

Provenance of each fixture:
  * qcp_kat.npz  -- the upstream MDAnalysisTests ``test_qcprot.py`` known-answer
    vector (7-atom Theobald example: coordinates, rmsd 0.719106, rotation),
    as quoted in SURVEY.md section 4 / Appendix A.4.  This is the only
    fixture whose expected values come from outside this repository.
  * synth_slice.npz -- float32 frames of the counter-based synthetic
    generator (oracle/synth.py), pinning the CPU<->GPU bit-identity contract.
  * c1_synth.npz, noalign_4096.npz, edges.npz -- expected outputs of the CPU
    oracle (oracle/rmsf_oracle.py, the numpy restatement of RMSF.py) on
    seeded synthetic inputs; inputs are stored as generator parameters
    (seed, shapes, selection, motion table) and regenerated bit-exactly.
The reference itself cannot run here (MDAnalysis / mpi4py absent), so these
oracle-derived vectors pin the oracle against drift and feed the GPU parity
tests; they are not reference outputs.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mdanalysis-mpi_amd"))

from oracle import rmsf_oracle as O  # noqa: E402
from oracle import synth as SY  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

# upstream test_qcprot.py
KAT_REF = np.array([[-2.803, -15.373, 24.556], [0.893, -16.062, 25.147], [1.368, -12.371, 25.885],
                    [-1.651, -12.153, 28.177], [-0.440, -15.218, 30.068], [2.551, -13.273, 31.372],
                    [0.105, -11.330, 33.567]])
KAT_MOB = np.array([[-14.739, -18.673, 15.040], [-12.473, -15.810, 16.074], [-14.802, -13.307, 14.408],
                    [-17.782, -14.852, 16.171], [-16.124, -14.617, 19.584], [-15.029, -11.037, 18.902],
                    [-18.577, -10.001, 17.996]])
KAT_RMSD = 0.719106
KAT_ROT = np.array([[0.72216358, -0.52038257, -0.45572112],
                    [0.69118937, 0.51700833, 0.50493528],
                    [-0.0271479, -0.67963547, 0.73304748]])


def motion_table(seed: int, n_frames: int, max_shift: float = 5.0) -> np.ndarray:
    # same recipe as rmsf_amd.synth.motion_table (kept local so the fixture
    # script does not import the product)
    rng = np.random.default_rng(seed)
    q = rng.standard_normal((n_frames, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    R = np.empty((n_frames, 3, 3))
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - z * w)
    R[:, 0, 2] = 2 * (x * z + y * w)
    R[:, 1, 0] = 2 * (x * y + z * w)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - x * w)
    R[:, 2, 0] = 2 * (x * z - y * w)
    R[:, 2, 1] = 2 * (y * z + x * w)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    t = 50.0 + rng.uniform(-max_shift, max_shift, (n_frames, 3))
    return np.ascontiguousarray(np.concatenate([R.reshape(n_frames, 9), t], axis=1))


def c1_inputs():
    seed, n_atoms, n_frames = 11, 3341, 98
    sel = np.sort(np.random.default_rng(12).choice(n_atoms, 214, replace=False))
    motion = motion_table(13, n_frames)
    masses = np.random.default_rng(14).uniform(1.0, 16.0, 214)
    return seed, n_atoms, n_frames, sel, motion, masses


def main():
    # 1. QCP known answer
    np.savez(os.path.join(OUT, "qcp_kat.npz"), ref=KAT_REF, mob=KAT_MOB, rmsd=KAT_RMSD, rot=KAT_ROT)

    # 2. generator slice (with and without rigid motion)
    mt = motion_table(3, 4)
    np.savez(os.path.join(OUT, "synth_slice.npz"), seed=5, n_atoms=100, frames=SY.frames(5, 100, 0, 4),
             motion=mt, frames_motion=SY.frames(5, 100, 0, 4, mt))

    # 3. C1-shaped case: 3341 atoms, 214 selected, 98 frames, random rigid motions
    seed, n_atoms, n_frames, sel, motion, masses = c1_inputs()
    traj = SY.frames(seed, n_atoms, 0, n_frames, motion)
    out = dict(seed=seed, n_atoms=n_atoms, n_frames=n_frames, sel=sel, motion=motion, masses=masses)
    for align, tag in ((None, "none"), ("frame0", "frame0"), ("average", "average")):
        for P in (1, 2, 8):
            r = O.rmsf_script(traj, sel, None, size=P, align=align)
            out[f"rmsf_{tag}_P{P}"] = r["rmsf"]
            if P == 1:
                out[f"mean_{tag}"] = r["mean"]
                out[f"m2_{tag}"] = r["m2"]
                if r["average"] is not None:
                    out["average"] = r["average"]
    r = O.rmsf_script(traj, sel, masses, size=2, align="average")
    out["rmsf_average_masses_P2"] = r["rmsf"]
    r = O.rmsf_script(traj, sel, None, size=1, align="average", start=3, stop=90, step=2)
    out["rmsf_average_slice"] = r["rmsf"]
    np.savez(os.path.join(OUT, "c1_synth.npz"), **out)

    # 4. no-alignment 4096 atoms x 1000 frames
    t2 = SY.frames(21, 4096, 0, 1000)
    np.savez(os.path.join(OUT, "noalign_4096.npz"), seed=21, n_atoms=4096, n_frames=1000,
             rmsf_P1=O.rmsf_script(t2, None, size=1, align=None)["rmsf"],
             rmsf_P3=O.rmsf_script(t2, None, size=3, align=None)["rmsf"])

    # 5. edges: one frame, identical frames, P > n_frames
    t3 = SY.frames(31, 50, 0, 3, motion_table(32, 3))
    ident = np.repeat(t3[:1], 10, axis=0)
    np.savez(os.path.join(OUT, "edges.npz"), seed=31, n_atoms=50, motion=motion_table(32, 3),
             one_frame=O.rmsf_script(t3[:1], None, size=1, align="average")["rmsf"],
             identical=O.rmsf_script(ident, None, size=1, align="average")["rmsf"],
             p8_of_3=O.rmsf_script(t3, None, size=8, align="average")["rmsf"],
             p1_of_3=O.rmsf_script(t3, None, size=1, align="average")["rmsf"])
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
