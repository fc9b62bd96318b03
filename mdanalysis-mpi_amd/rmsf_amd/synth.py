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


# Kurtosis of the generator's per-axis noise (a triangular law on
# [-sqrt(6), sqrt(6)], unit variance): E[g^4] = 2.4.
_NOISE_KURTOSIS = 2.4


def expected_rmsf(eng: Engine, n_atoms: int, seed: int = 0, a0: int = 0) -> torch.Tensor:
    """sqrt(3) sigma(a) for atoms a0..a0+n_atoms-1 (rmsf_synth_sigma, on the
    device): the population RMSF of the synthetic trajectory's atoms -- also
    after superposition, the noise being isotropic (rigid motions only
    rotate it)."""
    from ._lib import call

    s = eng.empty(n_atoms)
    call("rmsf_synth_sigma", s.data_ptr(), int(a0), int(n_atoms), int(seed), eng.stream)
    return s * np.sqrt(3.0)


def rmsf_sanity(eng: Engine, rmsf, n_frames: int, seed: int = 0, atoms=None, n_atoms: int | None = None,
                bound: float = 0.05) -> dict:
    """A result check that needs no reference implementation: every atom's
    RMSF against the generator's sqrt(3) sigma(a).  ``rmsf``: f64 [n_sel]
    (torch or numpy); ``atoms``: the selected atom indices (None = 0..n-1).
    The sampling spread of an n-frame RMSF is ~0.5 sqrt((k-1) / (3 n))
    relative (k = 2.4, the noise's kurtosis), so ``ok`` = max relative
    deviation below ``bound`` (5 %) or, for few frames, below 7 such spreads.
    Garbage frames (unwritten memory, a wrong stride, the wrong shard) miss
    by orders of magnitude."""
    r = torch.as_tensor(np.asarray(rmsf) if not isinstance(rmsf, torch.Tensor) else rmsf).to(eng.device,
                                                                                            torch.float64)
    if atoms is None:
        want = expected_rmsf(eng, n_atoms or r.numel(), seed)
    else:
        idx = torch.as_tensor(np.asarray(atoms, dtype=np.int64)).to(eng.device)
        want = expected_rmsf(eng, int(idx.max()) + 1, seed)[idx]
    if want.numel() != r.numel():
        raise ValueError("rmsf_sanity: one RMSF per atom expected")
    rel = (r / want - 1.0).abs()
    spread = 0.5 * float(np.sqrt((_NOISE_KURTOSIS - 1.0) / (3.0 * max(1, n_frames))))
    worst = float(rel.max()) if bool(torch.isfinite(rel).all()) else float("inf")
    return {"max_rel_dev": worst, "median_rel_dev": float(rel.median()), "expected_rel_spread": spread,
            "bound": max(bound, 7.0 * spread), "ok": worst < max(bound, 7.0 * spread),
            "rule": "|rmsf / (sqrt(3) sigma_gen) - 1| over every atom (rmsf_amd.synth.rmsf_sanity)"}
