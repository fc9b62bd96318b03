"""Golden vectors for RMSF.py:141-146's reduce order (generation-time only).

Like make_reference_vectors.py, this parses ``/root/reference/RMSF.py`` with
``ast`` and executes its statements unmodified -- here the exact=True path
(no alignment): each rank's Welford loop RMSF.py:137-138 over its block of
RMSF.py:66-69, its S of RMSF.py:140, and RMSF.py:146's RMSF of the reduced
Data.  The one thing supplied from outside is the ORDER in which
``comm.reduce(S, root=0, op=second_order_moments)`` (RMSF.py:143) applies
the reference's own ``second_order_moments`` (RMSF.py:36-41):

  * ``tree``: mpi4py's default object reduce (``rc.fast_reduce``,
    ``PyMPI_reduce_p2p``): a binomial tree, restated in
    oracle.rmsf_oracle.mpi4py_reduce from mpi4py's published source
    (mpi4py is not installed here: the order is upstream and unverified);
  * ``rank``: rank order (``rc.fast_reduce = False``: gather + _py_reduce).

At 4, 5 and 8 ranks the two orders give different bits; the generator
asserts that, so the vectors pin which one a build follows.

Also stored: RMSF.py:36-41 with an EMPTY first partial -- the reference's own
function on ((0, zeros, zeros), (3, mu, M)), whose mean is (3 mu) / 3, not mu
bit for bit.

Output: tests/golden/reduce_exec.npz.  Run from the repo root:
    python tests/golden/make_reduce_vectors.py
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, HERE]

from make_reference_vectors import REF, _compile  # noqa: E402
from oracle import rmsf_oracle as O  # noqa: E402  (mpi4py's tree order only)
from oracle import synth as SY  # noqa: E402

import ast  # noqa: E402

OUT = os.path.join(HERE, "reduce_exec.npz")


def load():
    tree = ast.parse(open(REF).read(), REF)
    fns = {}
    exec(_compile(tree, [36]), {"np": np}, fns)
    code = {
        "blocks": _compile(tree, [66, 67, 68, 69]),
        "sweep2": _compile(tree, [137, 138], {"select_atoms": "ts.positions[sel_idx]"}),
        "pack": _compile(tree, [140]),
        "final": _compile(tree, [146]),
    }
    return fns["second_order_moments"], code


def rank_states(code, traj, sel, size):
    """Each rank's S of RMSF.py:140 (RMSF.py:120-121, 137-138 unaligned)."""
    ns = dict(n_frames=traj.shape[0], size=size)
    exec(code["blocks"], ns)
    parts = []
    for b in ns["blocks"]:
        g = dict(np=np, sel_idx=sel, sumsquares=np.zeros((len(sel), 3)), start=b.start, stop=b.stop)
        g["mean"] = g["sumsquares"].copy()
        for k, frame in enumerate(range(b.start, b.stop)):
            g.update(ts=types.SimpleNamespace(positions=traj[frame].copy()), k=k)
            exec(code["sweep2"], g)
        exec(code["pack"], g)
        parts.append(g["S"])
    return parts


def final(code, Data):
    g = dict(np=np, Data=Data)
    exec(code["final"], g)
    return g["RMSF"]


def main():
    som, code = load()
    out = {}
    seed, n_atoms, nf = 23, 400, 77
    sel = np.arange(1, n_atoms, 2)
    traj = SY.frames(seed, n_atoms, 0, nf)
    out.update(seed=seed, n_atoms=n_atoms, n_frames=nf, sel=sel)
    for P in (2, 3, 4, 5, 8):
        parts = rank_states(code, traj, sel, P)
        for name, red in (("tree", O.mpi4py_reduce), ("rank", O.naive_reduce)):
            Data = red(parts, som)
            out[f"{name}_rmsf_P{P}"] = final(code, Data)
            out[f"{name}_mean_P{P}"] = Data[1]
            out[f"{name}_m2_P{P}"] = Data[2]
        differ = not (np.array_equal(out[f"tree_mean_P{P}"], out[f"rank_mean_P{P}"])
                      and np.array_equal(out[f"tree_m2_P{P}"], out[f"rank_m2_P{P}"]))
        if P <= 3:
            assert not differ, "the orders coincide up to 3 ranks"
        else:
            assert differ, f"P={P}: tree and rank order agree bit for bit; pick another input"
        print(f"P={P}: tree vs rank max |d rmsf| = "
              f"{np.abs(out[f'tree_rmsf_P{P}'] - out[f'rank_rmsf_P{P}']).max():.3e}")
    # RMSF.py:36-41 with an empty partial on either side
    rng = np.random.default_rng(5)
    mu = np.full((4, 3), 0.1)
    mu[1:] = rng.normal(30, 10, (3, 3))
    M = rng.uniform(0, 50, (4, 3))
    z = np.zeros((4, 3))
    T, m_a, q_a = som((0, z, z.copy()), (3, mu, M))
    T2, m_b, q_b = som((3, mu, M), (0, z, z.copy()))
    out.update(empty_mu=mu, empty_M=M, empty_left_mu=m_a, empty_left_M=q_a, empty_right_mu=m_b, empty_right_M=q_b)
    print("empty left: mu[0,0] =", repr(float(m_a[0, 0])), " (0.1 in, 3 frames)")
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
