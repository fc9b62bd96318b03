"""Device-backed ``CalcRMSDRotationalMatrix`` / ``get_rotation_matrix``.

Mirrors ``MDAnalysis.lib.qcprot.CalcRMSDRotationalMatrix(ref, conf, N, rot,
weights)`` as called at RMSF.py:48 (upstream Cython, not vendored in the
reference) and the script helper ``get_rotation_matrix`` (RMSF.py:43-51):
``rot`` (float64[9]) is filled in place and the rmsd is returned; the matrix
is applied to the mobile coordinates as ``conf @ rot.reshape(3, 3)``.

The per-frame pipeline never calls this -- it runs the same QCP solve inside
``rmsf_superpose`` for a whole block of frames -- but the single-structure
form is the FFI a user of the reference would reach for, and it carries the
upstream known-answer test.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call


def _as_f64_c(name: str, a, shape) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype != np.float64:
        raise ValueError(f"{name} must be float64, got {a.dtype}")  # upstream raises on wrong dtype
    a = np.ascontiguousarray(a)
    if shape is not None and a.shape != shape:
        raise ValueError(f"{name} must have shape {shape}, got {a.shape}")
    return a


def CalcRMSDRotationalMatrix(ref, conf, N: int, rot, weights=None) -> float:
    ref = _as_f64_c("ref", ref, (N, 3))
    conf = _as_f64_c("conf", conf, (N, 3))
    if not isinstance(rot, np.ndarray) or rot.dtype != np.float64 or rot.size != 9 or not rot.flags.c_contiguous:
        raise ValueError("rot must be a C-contiguous float64 array of 9 elements")
    w = None
    if weights is not None:
        w = _as_f64_c("weights", weights, (N,))
    rmsd = ctypes.c_double()
    call("rmsf_calc_rmsd_rotational_matrix", ref.ctypes.data, conf.ctypes.data, int(N), rot.ctypes.data,
         None if w is None else w.ctypes.data, ctypes.byref(rmsd))
    return rmsd.value


def get_rotation_matrix(ref_coordinates, mobile_coordinates, n_atoms: int) -> np.ndarray:
    """RMSF.py:43-51: the 3x3 optimal rotation (applied as ``x @ R``)."""
    rot = np.zeros(9, dtype=np.float64)
    CalcRMSDRotationalMatrix(ref_coordinates, mobile_coordinates, n_atoms, rot, weights=None)
    return rot.reshape(3, 3).copy()
