"""The rounding order of RMSF.py's rotation step (RMSF.py:100,134):
``ts.positions[:] = np.dot(ts.positions, R)`` promotes the float32 positions
to float64, multiplies by the f64 rotation through BLAS dgemm and stores
float32.  Whether the three products are summed fused or unfused can flip
the final f32 rounding.

CPU tier: on this host numpy's dot equals an FMA chain over a = 0, 1, 2
(``fma(p2, R2b, fma(p1, R1b, p0 R0b))``) bit for bit, and the unfused sum
only part of the time -- the kernel's ``apply_xform`` uses that chain
explicitly.  GPU tier: the device's transformed coordinates, run through
RMSF.py:99-101 on the host with the device's own per-frame rotation and
centre, are counted coordinate by coordinate: the number of f32 values that
differ is reported and must be 0.
"""
import os
from fractions import Fraction

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import synth as SY


def _fma(a: float, b: float, c: float) -> float:
    return float(Fraction(a) * Fraction(b) + Fraction(c))  # one rounding: fused multiply-add


def _chain(p: np.ndarray, R: np.ndarray) -> np.ndarray:
    return np.array([[_fma(r[2], R[2, b], _fma(r[1], R[1, b], r[0] * R[0, b])) for b in range(3)] for r in p])


def _unfused(p: np.ndarray, R: np.ndarray) -> np.ndarray:
    return (p[:, 0:1] * R[0] + p[:, 1:2] * R[1]) + p[:, 2:3] * R[2]


@pytest.fixture(scope="module")
def c1():
    ref = np.load(os.path.join(GOLDEN, "reference_exec.npz"))
    traj = SY.frames(int(ref["seed"]), int(ref["n_atoms"]), 0, int(ref["n_frames"]), ref["motion"])
    return ref, traj


def test_host_blas_dot_is_an_fma_chain(c1):
    ref, traj = c1
    rng = np.random.default_rng(0)
    q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    p = traj[5][ref["sel"]].astype(np.float64) - 50.0
    blas = np.dot(p, q)
    chain, unfused = _chain(p, q), _unfused(p, q)
    assert (blas == chain).all(), "numpy's dgemm no longer accumulates as an FMA chain on this host"
    print(f"\nnp.dot == FMA chain: {(blas == chain).mean():.3f}; == unfused sum: {(blas == unfused).mean():.3f}")


@pytest.mark.gpu
def test_device_transform_matches_rmsf_py_statements(c1):
    """Per-frame transformed f32 coordinates (the accumulate kernel in SUM
    mode with one frame per split returns exactly f64 of them) against
    RMSF.py:99-101 executed with numpy on the same positions, rotation and
    centres."""
    import torch

    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_XFORM_DOUBLES
    from rmsf_amd.engine import Engine

    ref, traj = c1
    sel = ref["sel"]
    nf, n_atoms, ns = traj.shape[0], traj.shape[1], len(sel)
    eng = Engine()
    d = torch.as_tensor(traj).to(eng.device)
    dsel = eng.sel_tensor(sel)
    refc, info = eng.reference_setup(ns, frame_ptr=d.data_ptr(), sel=dsel)
    xf = eng.empty(nf, RMSF_XFORM_DOUBLES)
    work = eng.empty(max(1, (eng.workspace_bytes(ns, nf) + 7) // 8))
    eng.superpose(d.data_ptr(), 3 * n_atoms, nf, ns, dsel, None, refc, info, xf, work)
    out = eng.empty(nf, 3 * ns)
    eng.accumulate(d.data_ptr(), 3 * n_atoms, nf, ns, dsel, xf, info, RMSF_MODE_SUM, nf, out, None)
    torch.cuda.synchronize()
    gpu = out.cpu().numpy().reshape(nf, ns, 3)
    xf, ref_com = xf.cpu().numpy(), info[:3].cpu().numpy()
    assert (gpu == gpu.astype(np.float32)).all()  # f64 of f32 values
    flips = flips_unfused = 0
    for f in range(nf):
        R, com = xf[f, :9].reshape(3, 3), xf[f, 9:12]
        positions = traj[f][sel].copy()
        positions[:] -= com                              # RMSF.py:99
        q = positions.astype(np.float64)
        positions[:] = np.dot(positions, R)              # RMSF.py:100
        positions += ref_com                             # RMSF.py:101
        flips += int((gpu[f].astype(np.float32) != positions).sum())
        alt = (_unfused(q, R).astype(np.float32).astype(np.float64) + ref_com).astype(np.float32)
        flips_unfused += int((alt != positions).sum())
    print(f"\nf32 coordinates differing from RMSF.py:99-101: device {flips} / {gpu.size}; "
          f"an unfused dot would give {flips_unfused}")
    assert flips == 0
