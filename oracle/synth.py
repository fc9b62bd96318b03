"""CPU regeneration of the synthetic trajectories -- TEST INFRASTRUCTURE ONLY.

Bit-identical restatement of ``k_synth`` (csrc/rmsf_kernels.hip) in numpy:
every float64 operation is one IEEE-rounded numpy op in the same order (no
FMA), so any (frame, atom) slice of the 24 GB device trajectories of configs
C2/C3 can be regenerated on the host for checking.
"""
from __future__ import annotations

import numpy as np

_MASK = (1 << 64) - 1
C_GOLD = np.uint64(0x9E3779B97F4A7C15)
C_M1 = np.uint64(0xBF58476D1CE4E5B9)
C_M2 = np.uint64(0x94D049BB133111EB)
C_STREAM = 0xD1B54A32D192ED03
TWO24 = 5.9604644775390625e-08
TWO53 = 1.1102230246251565e-16
SQRT6 = 2.449489742783178


def sm64(z):
    with np.errstate(over="ignore"):
        z = np.asarray(z, dtype=np.uint64) + C_GOLD
        z = (z ^ (z >> np.uint64(30))) * C_M1
        z = (z ^ (z >> np.uint64(27))) * C_M2
        return z ^ (z >> np.uint64(31))


def skey(seed: int, stream: int, i, j):
    s0 = np.uint64((int(seed) ^ ((stream * C_STREAM) & _MASK)) & _MASK)
    with np.errstate(over="ignore"):
        h = sm64(s0)
        h = sm64(h + np.asarray(i, dtype=np.uint64))
        return sm64(h + np.asarray(j, dtype=np.uint64))


def base_and_sigma(seed: int, atoms: np.ndarray):
    a = np.asarray(atoms, dtype=np.uint64)
    sigma = 0.2 + ((skey(seed, 2, a, 0) >> np.uint64(11)).astype(np.float64) * TWO53) * 1.8
    base = np.empty((len(a), 3))
    for c in range(3):
        base[:, c] = ((skey(seed, 1, a, c) >> np.uint64(11)).astype(np.float64) * TWO53) * 100.0
    return base, sigma


def frames(seed: int, n_atoms: int, f0: int, nf: int, motion: np.ndarray | None = None,
           atoms: np.ndarray | None = None) -> np.ndarray:
    """float32 [nf, len(atoms), 3]: frames f0..f0+nf-1 of the synthetic trajectory."""
    atoms = np.arange(n_atoms) if atoms is None else np.asarray(atoms)
    base, sigma = base_and_sigma(seed, atoms)
    a = atoms.astype(np.uint64)
    out = np.empty((nf, len(atoms), 3), dtype=np.float32)
    for fl in range(nf):
        f = f0 + fl
        p = np.empty((len(atoms), 3))
        for c in range(3):
            h = skey(seed, 3, np.uint64(f), np.uint64(3) * a + np.uint64(c))
            u = (h >> np.uint64(40)) + ((h >> np.uint64(16)) & np.uint64(0xFFFFFF))
            g = (u.astype(np.float64) * TWO24 - 1.0) * SQRT6
            s = sigma * g
            p[:, c] = base[:, c] + s
        if motion is not None:
            M = motion[f]
            d = p - 50.0
            for b in range(3):
                e0 = d[:, 0] * M[b]
                e1 = d[:, 1] * M[3 + b]
                e2 = d[:, 2] * M[6 + b]
                out[fl, :, b] = (((e0 + e1) + e2) + M[9 + b]).astype(np.float32)
        else:
            out[fl] = p.astype(np.float32)
    return out


def expected_rmsf(seed: int, atoms: np.ndarray) -> np.ndarray:
    """Population RMSF of the unaligned generator for infinitely many frames:
    sqrt(3) * sigma (unit-variance noise per axis)."""
    _, sigma = base_and_sigma(seed, atoms)
    return np.sqrt(3.0) * sigma
