"""Synthetic trajectories generated directly in HBM.

The device generator (``rmsf_synth_frames`` / ``k_synth``) is counter based:
frame f, atom a, axis c of seed s is a pure function of (s, f, a, c), so any
slice can be regenerated on the host for checking and each rank of a sharded
run generates only its own frames.  Rigid motions for config C3 come from a
small host table [n_frames, 12] (R row-major, t) uploaded once.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import Engine


def motion_table(seed: int, n_frames: int, max_shift: float = 5.0) -> np.ndarray:
    """Uniform random rotations (normalised Gaussian quaternions) and
    translations of +-max_shift about the box centre (50, 50, 50)."""
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


def generate(eng: Engine, n_atoms: int, f0: int, nf: int, seed: int = 0, motion: np.ndarray | None = None,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """float32 [nf, n_atoms, 3] in HBM: frames f0..f0+nf-1 of the synthetic
    trajectory (``motion`` indexed by global frame)."""
    if out is None:
        out = eng.empty(nf, n_atoms, 3, dtype=torch.float32)
    m = None
    if motion is not None:
        m = torch.as_tensor(np.ascontiguousarray(motion, dtype=np.float64)).to(eng.device)
    eng.synth_frames(out, n_atoms, f0, nf, seed, m, fstride=out.stride(0))
    return out
