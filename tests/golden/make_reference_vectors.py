"""Golden vectors from the reference's OWN statements (generation-time only).

``/root/reference/RMSF.py`` cannot be imported here: its module-level imports
need MDAnalysis and mpi4py, neither of which is installed (ordinary
``ModuleNotFoundError``; no permission denial).  Its hot-path arithmetic,
however, is plain numpy written in the script itself.  This generator parses
RMSF.py with ``ast`` (at generation time; nothing of it is stored), picks the
statements listed below by line number and executes them **unmodified**, with
three kinds of inputs supplied from outside because they live in absent
dependencies:

  * trajectory frames and the CA selection (MDAnalysis readers/selections):
    seeded synthetic float32 frames (oracle/synth.py) and a fixed index set;
    the three AtomGroup ``.positions`` reads are rewritten to
    ``ts.positions[sel_idx]`` / the reference rows -- what upstream
    ``AtomGroup.positions`` returns (a fancy-indexed copy of the Timestep);
  * ``AtomGroup.center_of_mass()`` (RMSF.py:84,94,117,127): upstream
    ``AtomGroup.center(weights=masses)`` restated as
    ``einsum('ij,ij->j', x, m[:, None]) / m.sum()`` (upstream formula,
    unpinned version);
  * ``qcprot.CalcRMSDRotationalMatrix`` (called by the reference's own
    ``get_rotation_matrix``, RMSF.py:43-51): oracle.rmsf_oracle's QCP, which is
    pinned by the upstream test_qcprot.py known answer (tests/golden/qcp_kat.npz).

MPI is emulated by running the ranks of the block decomposition the
reference's own lines 66-69 produce, one after another; ``Allreduce(SUM)``
(RMSF.py:110) is the rank-ordered sum and ``comm.reduce(op=...)`` (RMSF.py:143)
folds the reference's own ``second_order_moments`` in rank order.

Executed reference statements (RMSF.py line numbers):
  36-41 second_order_moments   43-51 get_rotation_matrix   66-69 blocks
  85 (ref centring)  95, 97, 99-101, 103 (sweep 1)  105, 111 (average)
  118 (pass-2 reference)  128, 131, 133-135, 137-138 (sweep 2)  140 (S)  146 (RMSF)

Every atom of the frame is transformed (RMSF.py:99-101 acts on all atoms), so
these vectors also check that restricting the work to the selection (the
build's SURVEY Q3 disposition) is exact.

RMSF.py:113 wraps the f64 average in a MemoryReader Universe; whether that
reader keeps f64 or casts to float32 is an upstream detail not pinned here
(MDAnalysis is absent).  Every end-to-end case is therefore run under both
readings: the f64 one (keys without suffix) and the float32 one (``_avg32``:
the average cast to float32 before lines 116-118).

Output: tests/golden/reference_exec.npz (inputs as generator parameters, the
reference's outputs) and tests/golden/reference_literal.npz (RMSF.py's own
input shape -- 47,681 atoms, 214 CA, 10 frames under ``mpirun -n 2`` -- and
the same at 2 and 4 frames).  Run from the repo root:
    python tests/golden/make_reference_vectors.py [literal]
"""
from __future__ import annotations

import ast
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import rmsf_oracle as O  # noqa: E402  (QCP only, KAT-pinned)
from oracle import synth as SY  # noqa: E402

REF = "/root/reference/RMSF.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_exec.npz")


class _Subst(ast.NodeTransformer):
    """Replace ``<name>.select_atoms(...).positions`` / ``<name>.positions``
    AtomGroup reads by a plain expression (see module docstring)."""

    def __init__(self, table):
        self.table = table

    def visit_Attribute(self, node):
        self.generic_visit(node)
        if node.attr == "positions":
            v = node.value
            if isinstance(v, ast.Call) and isinstance(v.func, ast.Attribute) and v.func.attr == "select_atoms":
                key = "select_atoms"
            elif isinstance(v, ast.Name):
                key = v.id
            else:
                return node
            if key in self.table:
                return ast.copy_location(ast.parse(self.table[key], mode="eval").body, node)
        return node


def _statements(tree, lines):
    found = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.stmt) and getattr(node, "lineno", None) in lines:
            found[node.lineno] = node
    missing = sorted(set(lines) - set(found))
    if missing:
        raise SystemExit(f"RMSF.py statements not found at lines {missing}")
    return [found[n] for n in lines]


def _compile(tree, lines, subst=None):
    body = _statements(tree, lines)
    if subst:
        body = [_Subst(subst).visit(ast.fix_missing_locations(ast.parse(ast.unparse(s)).body[0])) for s in body]
    mod = ast.fix_missing_locations(ast.Module(body=body, type_ignores=[]))
    return compile(mod, f"{REF}:{lines[0]}-{lines[-1]}", "exec")


def load_reference():
    tree = ast.parse(open(REF).read(), REF)
    fns = {}
    exec(_compile(tree, [36, 43]), {"np": np, "qcp": types.SimpleNamespace(
        CalcRMSDRotationalMatrix=O.CalcRMSDRotationalMatrix)}, fns)
    code = {
        "blocks": _compile(tree, [66, 67, 68, 69]),
        "ref": _compile(tree, [85], {"ref_atoms": "ref_positions"}),
        "sweep1": _compile(tree, [95, 97, 99, 100, 101, 103], {"mobile_atoms": "ts.positions[sel_idx]"}),
        "average": _compile(tree, [105]),
        "divide": _compile(tree, [111]),
        "ref2": _compile(tree, [118], {"ref_atoms": "ref_positions"}),
        "sweep2": _compile(tree, [128, 131, 133, 134, 135, 137, 138],
                           {"mobile_atoms": "ts.positions[sel_idx]", "select_atoms": "ts.positions[sel_idx]"}),
        "pack": _compile(tree, [140]),
        "final": _compile(tree, [146]),
    }
    return fns, code


def com_upstream(x, m):
    """MDAnalysis AtomGroup.center(weights=masses) (upstream; unpinned)."""
    return np.einsum("ij,ij->j", x, m[:, None]) / m.sum()


def run_reference(fns, code, traj, sel, masses, size, avg_f32=False):
    """RMSF.py for ``mpirun -n size`` on a synthetic trajectory (all atoms).
    ``avg_f32``: the MemoryReader of RMSF.py:113 taken to store float32."""
    n_frames, n_all = traj.shape[:2]
    ns = dict(np=np, n_frames=n_frames, size=size)
    exec(code["blocks"], ns)
    blocks = ns["blocks"]

    g = dict(np=np, get_rotation_matrix=fns["get_rotation_matrix"], sel_idx=sel,
             mobile_atoms=types.SimpleNamespace(n_atoms=len(sel)))  # only .n_atoms is read (RMSF.py:97,131)
    # RMSF.py:80-87: frame 0 of the reference copy
    g["ref_positions"] = traj[0][sel].copy()
    g["ref_com"] = com_upstream(g["ref_positions"], masses).astype(np.float64)
    exec(code["ref"], g)
    ref_coordinates, ref_com = g["ref_coordinates"], g["ref_com"]

    # sweep 1 per rank (RMSF.py:89-105), then Allreduce(SUM) in rank order
    sums = []
    for b in blocks:
        g.update(pos=np.zeros((n_all, 3)), ref_coordinates=ref_coordinates, ref_com=ref_com)
        for frame in range(b.start, b.stop):
            ts = types.SimpleNamespace(positions=traj[frame].copy())  # Timestep: float32 [n_all, 3]
            g["ts"] = ts
            g["mobile_com"] = com_upstream(ts.positions[sel], masses).astype(np.float64)
            exec(code["sweep1"], g)
        exec(code["average"], g)
        sums.append(g["pos"])
    total = np.zeros(n_all * 3)
    for s in sums:
        total += s
    g.update(positions=total, n_frames=n_frames)
    exec(code["divide"], g)
    average = g["positions"].reshape(-1, 3)

    # pass-2 reference (RMSF.py:113-118): the MemoryReader rows of the CA
    # (f64, or float32 under the other reading of :113)
    g["ref_positions"] = average[sel].astype(np.float32) if avg_f32 else average[sel]
    g["ref_com"] = com_upstream(g["ref_positions"], masses).astype(np.float64)
    exec(code["ref2"], g)
    ref_coordinates, ref_com = g["ref_coordinates"], g["ref_com"]

    # sweep 2 per rank (RMSF.py:120-140)
    parts = []
    for b in blocks:
        g.update(sumsquares=np.zeros((len(sel), 3)), ref_coordinates=ref_coordinates, ref_com=ref_com,
                 start=b.start, stop=b.stop)
        g["mean"] = g["sumsquares"].copy()
        for k, frame in enumerate(range(b.start, b.stop)):
            ts = types.SimpleNamespace(positions=traj[frame].copy())
            g.update(ts=ts, k=k)
            g["mobile_com"] = com_upstream(ts.positions[sel], masses).astype(np.float64)
            exec(code["sweep2"], g)
        exec(code["pack"], g)
        parts.append(g["S"])

    # comm.reduce(S, root=0, op=second_order_moments): rank-order fold
    Data = parts[0]
    for S in parts[1:]:
        Data = fns["second_order_moments"](Data, S)
    g["Data"] = Data
    exec(code["final"], g)
    return dict(rmsf=g["RMSF"], mean=Data[1], m2=Data[2], n=Data[0], average=average[sel],
                blocks=np.array([[b.start, b.stop] for b in blocks]))


def main():
    fns, code = load_reference()
    out = {}

    # RMSF.py:66-69 on a grid of (n_frames, size)
    grid = [(n, p) for n in (0, 1, 2, 3, 7, 10, 98, 1000, 20000) for p in (1, 2, 3, 4, 7, 8, 16)]
    tab = []
    for n, p in grid:
        ns = dict(n_frames=n, size=p)
        exec(code["blocks"], ns)
        for r, b in enumerate(ns["blocks"]):
            tab.append((n, p, r, b.start, b.stop))
    out["blocks"] = np.array(tab, dtype=np.int64)

    # RMSF.py:36-41 on random partials (integer counts, as S[0] = stop - start)
    rng = np.random.default_rng(41)
    n1 = rng.integers(1, 5000, 16)
    n2 = rng.integers(1, 5000, 16)
    mu1, mu2 = rng.normal(50, 20, (2, 16, 10, 3))
    M1, M2 = rng.uniform(0, 1e4, (2, 16, 10, 3))
    T, mu, M = zip(*[fns["second_order_moments"]((int(n1[i]), mu1[i], M1[i]), (int(n2[i]), mu2[i], M2[i]))
                     for i in range(16)])
    out.update(chan_n1=n1, chan_n2=n2, chan_mu1=mu1, chan_mu2=mu2, chan_M1=M1, chan_M2=M2,
               chan_T=np.array(T), chan_mu=np.array(mu), chan_M=np.array(M))

    # RMSF.py end to end on a C1-shaped synthetic trajectory
    seed, n_atoms, n_frames = 11, 3341, 98
    sel = np.sort(np.random.default_rng(12).choice(n_atoms, 214, replace=False))
    from make_golden import motion_table

    motion = motion_table(13, n_frames)
    traj = SY.frames(seed, n_atoms, 0, n_frames, motion)
    ca = np.full(len(sel), 12.011)  # CA masses (uniform, as for the reference's selection)
    het = np.random.default_rng(14).uniform(1.0, 16.0, len(sel))
    out.update(seed=seed, n_atoms=n_atoms, n_frames=n_frames, sel=sel, motion=motion, masses_ca=ca, masses_het=het)
    for tag, m in (("ca", ca), ("het", het)):
        for P in (1, 2, 3):
            r = run_reference(fns, code, traj, sel, m, P)
            out[f"rmsf_{tag}_P{P}"] = r["rmsf"]
            if P == 1:
                out[f"mean_{tag}"] = r["mean"]
                out[f"m2_{tag}"] = r["m2"]
                out[f"average_{tag}"] = r["average"]
            r32 = run_reference(fns, code, traj, sel, m, P, avg_f32=True)
            out[f"rmsf_{tag}_P{P}_avg32"] = r32["rmsf"]
            if P == 1:
                out[f"mean_{tag}_avg32"] = r32["mean"]
            print(f"masses={tag} P={P}: n={r['n']} blocks={r['blocks'].tolist()} "
                  f"rmsf[:3]={r['rmsf'][:3]} |f64 - f32 reading| max {np.abs(r['rmsf'] - r32['rmsf']).max():.3e}")

    # 100k atoms x 256 frames (all atoms selected, uniform masses), both
    # readings of RMSF.py:113; 2,048 sampled rows stored (each atom's RMSF
    # depends on the others only through the per-frame rotations)
    bseed, bn, bf = 21, 100_000, 256
    bmotion = motion_table(22, bf)
    btraj = SY.frames(bseed, bn, 0, bf, bmotion)
    bsel = np.arange(bn)
    bm = np.full(bn, 12.011)
    rows = np.sort(np.random.default_rng(23).choice(bn, 2048, replace=False))
    b64 = run_reference(fns, code, btraj, bsel, bm, 1)
    b32 = run_reference(fns, code, btraj, bsel, bm, 1, avg_f32=True)
    gap = np.abs(b64["rmsf"] - b32["rmsf"])
    out.update(big_seed=bseed, big_n_atoms=bn, big_n_frames=bf, big_motion=bmotion, big_rows=rows,
               big_rmsf=b64["rmsf"][rows], big_rmsf_avg32=b32["rmsf"][rows], big_average=b64["average"][rows],
               big_gap_max=gap.max(), big_gap_mean=gap.mean())
    print(f"100k x 256: |f64 - f32 reading| max {gap.max():.3e} mean {gap.mean():.3e}")
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


# RMSF.py's literal input shape (RMSF.py:34,56: GRO/XTC = adk_oplsaa, 47,681
# atoms, 214 CA, 10 frames, run as ``mpirun -n 2``: 5 frames per rank --
# upstream facts) on synthetic frames, and the same shape at
# 2 and 4 frames: the few-frame end where one f32 rounding flip of an aligned
# coordinate weighs most (|x - mean| ulp / (N RMSF)).
OUT_LITERAL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_literal.npz")
LITERAL = dict(seed=61, n_atoms=47_681, n_sel=214, frames=(2, 4, 10), sizes=(1, 2), sel_seed=62, motion_seed=63)


def main_literal():
    from make_golden import motion_table

    fns, code = load_reference()
    L = LITERAL
    sel = np.sort(np.random.default_rng(L["sel_seed"]).choice(L["n_atoms"], L["n_sel"], replace=False))
    ca = np.full(len(sel), 12.011)  # CA masses (every selected atom a carbon, as for the reference's selection)
    out = dict(seed=L["seed"], n_atoms=L["n_atoms"], sel=sel, masses=ca, frames=np.array(L["frames"]),
               sizes=np.array(L["sizes"]))
    nmax = max(L["frames"])
    motion = motion_table(L["motion_seed"], nmax)
    out["motion"] = motion
    traj_all = SY.frames(L["seed"], L["n_atoms"], 0, nmax, motion)
    for nf in L["frames"]:
        traj = traj_all[:nf]  # the first nf frames of one trajectory
        for P in L["sizes"]:
            r = run_reference(fns, code, traj, sel, ca, P)
            for k in ("rmsf", "mean", "m2", "average"):
                out[f"{k}_F{nf}_P{P}"] = r[k]
            out[f"blocks_F{nf}_P{P}"] = r["blocks"]
            print(f"literal shape, {nf} frames, P={P}: blocks={r['blocks'].tolist()} rmsf[:3]={r['rmsf'][:3]}")
    np.savez_compressed(OUT_LITERAL, **out)
    print("wrote", OUT_LITERAL)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if sys.argv[1:] == ["literal"]:
        main_literal()
    else:
        main()
        main_literal()
