"""CPU ORACLE for the frame-parallel RMSF path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the
reported CPU baseline.  The product (``mdanalysis-mpi_amd/rmsf_amd``) never
imports it and has no CPU fallback.

What it restates (numpy, the same statements the reference executes):
  * /root/reference/RMSF.py:36-41  ``second_order_moments``     -> second_order_moments
  * RMSF.py:43-51                  ``get_rotation_matrix``      -> get_rotation_matrix
  * RMSF.py:59-72                  frame blocks per rank       -> block_ranges
  * RMSF.py:80-87                  frame-0 reference            -> centred_reference
  * RMSF.py:89-105                 sweep 1 (align + sum)        -> rank_sweep1
  * RMSF.py:107-118                Allreduce / average / ref    -> rmsf_script
  * RMSF.py:120-140                sweep 2 (align + Welford)    -> rank_sweep2
  * RMSF.py:141-146                reduce + finalise            -> rmsf_script
  * MDAnalysis.lib.qcprot (upstream Cython, NOT vendored and NOT installed
    here; restated from the published QCP algorithm -- Theobald 2005, Liu et
    al. 2010 -- as SURVEY.md Appendix A.1-A.3 spells it)  -> inner_product,
    fast_calc_rmsd_and_rotation, CalcRMSDRotationalMatrix
  * MDAnalysis ``AtomGroup.center_of_mass`` (upstream, not vendored):
    sum(x * m) / sum(m) in float64                            -> center_of_mass

Parity pinning (see DESIGN.md "Oracle"):
  * QCP is pinned by the upstream ``test_qcprot.py`` known-answer vector
    (rmsd 0.719106, the rotation matrix) quoted in SURVEY.md section 4 / A.4,
    and cross-checked against an independent Kabsch SVD.
  * Welford / Chan / finalise are pinned by analytic known answers and by an
    independent two-pass numpy variance.
  * The end-to-end RMSF of RMSF.py on real MDAnalysis data is UNPINNED: the
    reference cannot run here (MDAnalysis, mpi4py and MDAnalysisTests data
    are not installed; no network), so no reference output exists.
"""
from __future__ import annotations

import math

import numpy as np

# ---------------------------------------------------------------------------
# RMSF.py:59-72


def block_ranges(n_frames: int, size: int) -> list[range]:
    """RMSF.py:63-69 verbatim semantics."""
    n_blocks = size
    n_frames_per_block = n_frames // n_blocks
    blocks = [range(i * n_frames_per_block, (i + 1) * n_frames_per_block) for i in range(n_blocks - 1)]
    blocks.append(range((n_blocks - 1) * n_frames_per_block, n_frames))
    return blocks


# ---------------------------------------------------------------------------
# MDAnalysis center_of_mass (RMSF.py:84,94,117,127)


def center_of_mass(pos: np.ndarray, masses: np.ndarray | None = None) -> np.ndarray:
    m = np.ones(len(pos), dtype=np.float64) if masses is None else np.asarray(masses, dtype=np.float64)
    return (pos * m[:, None]).sum(axis=0) / m.sum()


# ---------------------------------------------------------------------------
# qcprot (RMSF.py:48)


def _seq_sum(terms: np.ndarray) -> float:
    """terms[0] + terms[1] + ... added one at a time from 0.0, as a C loop
    ``G += term`` does (np.cumsum accumulates sequentially; ndarray.sum()
    would sum pairwise)."""
    return float(np.cumsum(terms)[-1]) if len(terms) else 0.0


def inner_product(ref: np.ndarray, conf: np.ndarray, weights=None):
    """qcprot InnerProduct(A, conf, ref, N, weights): A[a][b] = sum w conf_a ref_b,
    E0 = (G1 + G2) * 0.5.  Returns (A[9] list, E0).

    Summation order of the published qcprot loop (Theobald's qcprot.c
    ``InnerProduct``, which MDAnalysis.lib.qcprot restates in Cython --
    upstream, not vendored or installed here, so unverified in this
    container): ONE pass over the atoms i = 0..N-1, every accumulator updated
    per atom in turn --
        x1 = w conf_x (y1, z1 alike)        (x1 = conf_x without weights)
        G1 += x1 conf_x + y1 conf_y + z1 conf_z
        G2 += w (ref_x^2 + ref_y^2 + ref_z^2)   (without the w factor unweighted)
        A[3a + b] += (a1 ref_b)
    each right-hand side evaluated left to right and rounded per operation
    (no contraction), then added to the running sum.  The axis-0 reduction
    of an [N, 3, 3] product array is sequential in numpy, so A follows that
    order; G1/G2's per-atom terms are summed by ``_seq_sum``."""
    conf = np.asarray(conf, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if weights is None:
        wc = conf
        g1 = (conf[:, 0] * conf[:, 0] + conf[:, 1] * conf[:, 1]) + conf[:, 2] * conf[:, 2]
        g2 = (ref[:, 0] * ref[:, 0] + ref[:, 1] * ref[:, 1]) + ref[:, 2] * ref[:, 2]
    else:
        w = np.asarray(weights, dtype=np.float64)
        wc = conf * w[:, None]
        g1 = (wc[:, 0] * conf[:, 0] + wc[:, 1] * conf[:, 1]) + wc[:, 2] * conf[:, 2]
        g2 = w * ((ref[:, 0] * ref[:, 0] + ref[:, 1] * ref[:, 1]) + ref[:, 2] * ref[:, 2])
    A = (wc[:, :, None] * ref[:, None, :]).sum(axis=0).reshape(9)
    G1, G2 = _seq_sum(g1), _seq_sum(g2)
    return [float(v) for v in A], (G1 + G2) * 0.5


def _div(a: float, b: float) -> float:
    """IEEE double division (C semantics: x/0 -> inf or nan, no exception)."""
    with np.errstate(all="ignore"):
        return float(np.float64(a) / np.float64(b))


def fast_calc_rmsd_and_rotation(A, E0: float, N: float):
    """qcprot FastCalcRMSDAndRotation (minScore < 0): returns (rot[9], rmsd, iters).

    Scalar IEEE-double restatement of the published algorithm, same operation
    sequence as SURVEY.md Appendix A.2-A.3."""
    Sxx, Sxy, Sxz, Syx, Syy, Syz, Szx, Szy, Szz = (float(v) for v in A)
    Sxx2, Syy2, Szz2 = Sxx * Sxx, Syy * Syy, Szz * Szz
    Sxy2, Syz2, Sxz2 = Sxy * Sxy, Syz * Syz, Sxz * Sxz
    Syx2, Szy2, Szx2 = Syx * Syx, Szy * Szy, Szx * Szx
    SyzSzymSyySzz2 = 2.0 * (Syz * Szy - Syy * Szz)
    Sxx2Syy2Szz2Syz2Szy2 = Syy2 + Szz2 - Sxx2 + Syz2 + Szy2
    C2 = -2.0 * (Sxx2 + Syy2 + Szz2 + Sxy2 + Syx2 + Sxz2 + Szx2 + Syz2 + Szy2)
    C1 = 8.0 * (Sxx * Syz * Szy + Syy * Szx * Sxz + Szz * Sxy * Syx - Sxx * Syy * Szz - Syz * Szx * Sxy
                - Szy * Syx * Sxz)
    SxzpSzx, SyzpSzy, SxypSyx = Sxz + Szx, Syz + Szy, Sxy + Syx
    SyzmSzy, SxzmSzx, SxymSyx = Syz - Szy, Sxz - Szx, Sxy - Syx
    SxxpSyy, SxxmSyy = Sxx + Syy, Sxx - Syy
    Sxy2Sxz2Syx2Szx2 = Sxy2 + Sxz2 - Syx2 - Szx2
    C0 = (Sxy2Sxz2Syx2Szx2 * Sxy2Sxz2Syx2Szx2
          + (Sxx2Syy2Szz2Syz2Szy2 + SyzSzymSyySzz2) * (Sxx2Syy2Szz2Syz2Szy2 - SyzSzymSyySzz2)
          + (-(SxzpSzx) * (SyzmSzy) + (SxymSyx) * (SxxmSyy - Szz))
          * (-(SxzmSzx) * (SyzpSzy) + (SxymSyx) * (SxxmSyy + Szz))
          + (-(SxzpSzx) * (SyzpSzy) - (SxypSyx) * (SxxpSyy - Szz))
          * (-(SxzmSzx) * (SyzmSzy) - (SxypSyx) * (SxxpSyy + Szz))
          + (+(SxypSyx) * (SyzpSzy) + (SxzpSzx) * (SxxmSyy + Szz))
          * (-(SxymSyx) * (SyzmSzy) + (SxzpSzx) * (SxxpSyy + Szz))
          + (+(SxypSyx) * (SyzmSzy) + (SxzmSzx) * (SxxmSyy - Szz))
          * (-(SxymSyx) * (SyzpSzy) + (SxzmSzx) * (SxxpSyy - Szz)))
    lam = float(E0)
    iters = 0
    for i in range(50):
        iters = i + 1
        old = lam
        x2 = lam * lam
        b = (x2 + C2) * lam
        a = b + C1
        delta = _div(a * lam + C0, 2.0 * x2 * lam + b + a)
        lam -= delta
        if abs(lam - old) < abs(1e-11 * lam):  # False for NaN, as in C
            break
    rmsd = math.sqrt(abs(_div(2.0 * (E0 - lam), N)))

    a11, a12, a13, a14 = SxxpSyy + Szz - lam, SyzmSzy, -SxzmSzx, SxymSyx
    a21, a22, a23, a24 = SyzmSzy, SxxmSyy - Szz - lam, SxypSyx, SxzpSzx
    a31, a32, a33, a34 = a13, a23, Syy - Sxx - Szz - lam, SyzpSzy
    a41, a42, a43, a44 = a14, a24, a34, Szz - SxxpSyy - lam
    a3344_4334 = a33 * a44 - a43 * a34
    a3244_4234 = a32 * a44 - a42 * a34
    a3243_4233 = a32 * a43 - a42 * a33
    a3143_4133 = a31 * a43 - a41 * a33
    a3144_4134 = a31 * a44 - a41 * a34
    a3142_4132 = a31 * a42 - a41 * a32
    q1 = a22 * a3344_4334 - a23 * a3244_4234 + a24 * a3243_4233
    q2 = -a21 * a3344_4334 + a23 * a3144_4134 - a24 * a3143_4133
    q3 = a21 * a3244_4234 - a22 * a3144_4134 + a24 * a3142_4132
    q4 = -a21 * a3243_4233 + a22 * a3143_4133 - a23 * a3142_4132
    qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4
    evecprec = 1e-6
    if qsqr < evecprec:
        q1 = a12 * a3344_4334 - a13 * a3244_4234 + a14 * a3243_4233
        q2 = -a11 * a3344_4334 + a13 * a3144_4134 - a14 * a3143_4133
        q3 = a11 * a3244_4234 - a12 * a3144_4134 + a14 * a3142_4132
        q4 = -a11 * a3243_4233 + a12 * a3143_4133 - a13 * a3142_4132
        qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4
        if qsqr < evecprec:
            a1324_1423 = a13 * a24 - a14 * a23
            a1224_1422 = a12 * a24 - a14 * a22
            a1223_1322 = a12 * a23 - a13 * a22
            a1124_1421 = a11 * a24 - a14 * a21
            a1123_1321 = a11 * a23 - a13 * a21
            a1122_1221 = a11 * a22 - a12 * a21
            q1 = a42 * a1324_1423 - a43 * a1224_1422 + a44 * a1223_1322
            q2 = -a41 * a1324_1423 + a43 * a1124_1421 - a44 * a1123_1321
            q3 = a41 * a1224_1422 - a42 * a1124_1421 + a44 * a1122_1221
            q4 = -a41 * a1223_1322 + a42 * a1123_1321 - a43 * a1122_1221
            qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4
            if qsqr < evecprec:
                q1 = a32 * a1324_1423 - a33 * a1224_1422 + a34 * a1223_1322
                q2 = -a31 * a1324_1423 + a33 * a1124_1421 - a34 * a1123_1321
                q3 = a31 * a1224_1422 - a32 * a1124_1421 + a34 * a1122_1221
                q4 = -a31 * a1223_1322 + a32 * a1123_1321 - a33 * a1122_1221
                qsqr = q1 * q1 + q2 * q2 + q3 * q3 + q4 * q4
                if qsqr < evecprec:
                    return [1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0], rmsd, iters
    normq = math.sqrt(qsqr) if qsqr == qsqr else math.nan
    q1, q2, q3, q4 = _div(q1, normq), _div(q2, normq), _div(q3, normq), _div(q4, normq)
    a2, x2, y2, z2 = q1 * q1, q2 * q2, q3 * q3, q4 * q4
    xy, az, zx, ay, yz, ax = q2 * q3, q1 * q4, q4 * q2, q1 * q3, q3 * q4, q1 * q2
    rot = [a2 + x2 - y2 - z2, 2 * (xy + az), 2 * (zx - ay),
           2 * (xy - az), a2 - x2 + y2 - z2, 2 * (yz + ax),
           2 * (zx + ay), 2 * (yz - ax), a2 - x2 - y2 + z2]
    return rot, rmsd, iters


def CalcRMSDRotationalMatrix(ref, conf, N, rot, weights=None) -> float:
    """qcprot.CalcRMSDRotationalMatrix: fills rot (f64[9]) in place, returns rmsd."""
    A, E0 = inner_product(ref, conf, weights)
    r, rmsd, _ = fast_calc_rmsd_and_rotation(A, E0, float(N))
    rot[:] = r
    return rmsd


def get_rotation_matrix(ref_coordinates, mobile_coordinates, n_atoms):
    """RMSF.py:43-51."""
    rotation_matrix = np.zeros(9, dtype=np.float64)
    CalcRMSDRotationalMatrix(ref_coordinates, mobile_coordinates, n_atoms, rotation_matrix, weights=None)
    return rotation_matrix.reshape(3, 3).copy()


# ---------------------------------------------------------------------------
# RMSF.py:36-41


def second_order_moments(S1, S2):
    T = S1[0] + S2[0]
    mu = (S1[0] * S1[1] + S2[0] * S2[1]) / T
    M = S1[2] + S2[2] + (S1[0] * S2[0] / T) * (S2[1] - S1[1]) ** 2
    return T, mu, M


def _op_or_skip(S1, S2):
    """second_order_moments, except where RMSF.py:39 raises (two empty
    states, T = 0): the build continues with the empty state instead."""
    if S1[0] + S2[0] == 0:
        return S1
    return second_order_moments(S1, S2)


def _empty_as_zeros(S):
    """An empty rank's S is (0, zeros, zeros) (RMSF.py:119-121 with no frame);
    whatever arrays a caller passes for it are replaced by those zeros."""
    if S[0] == 0:
        z = np.zeros_like(np.asarray(S[1], dtype=np.float64))
        return (0, z, z.copy())
    return S


def mpi4py_reduce(parts, op):
    """mpi4py's lowercase ``comm.reduce(sendobj, op=op, root=0)`` as RMSF.py:143
    calls it, evaluated for every rank at once: ``parts[r]`` is rank r's
    ``sendobj``; returns rank 0's result.

    Restated from mpi4py's published ``msgpickle.pxi`` (upstream, NOT vendored
    or installed here, so unverified in this container): with
    ``mpi4py.rc.fast_reduce`` (its default) an intracommunicator's object
    reduce is ``PyMPI_reduce_p2p`` -- each rank starts from a copy of its own
    object; for mask = 1, 2, 4, ...: a rank with the mask bit set sends its
    result to ``rank & ~mask`` and is done; otherwise it receives from
    ``rank | mask`` (when that rank exists) and computes
    ``result = op(result, received)``.  Rank 0 ends with the result (and
    forwards it to root when root != 0, which does not change it)."""
    result = list(parts)
    size = len(result)
    mask = 1
    while mask < size:
        for r in range(0, size, 2 * mask):  # the ranks still receiving at this mask
            if r + mask < size:
                result[r] = op(result[r], result[r + mask])
        mask <<= 1
    return result[0]


def naive_reduce(parts, op):
    """mpi4py's object reduce with ``rc.fast_reduce = False`` (a gather to
    root, then ``_py_reduce``): ``res = parts[0]; res = op(res, parts[i])``
    in rank order."""
    res = parts[0]
    for S in parts[1:]:
        res = op(res, S)
    return res


MERGE_ORDERS = ("mpi4py", "rank")


def chan_fold(parts, order: str = "mpi4py"):
    """RMSF.py:143 ``comm.reduce(S, root=0, op=second_order_moments)`` over the
    ranks' S (rank order in ``parts``), applying the op in mpi4py's order
    (``"mpi4py"``: the default binomial tree, ``mpi4py_reduce``; ``"rank"``:
    rank order, ``naive_reduce``).  Empty ranks are RMSF.py's (0, zeros,
    zeros) and enter the op like any other; a merge of two empty states
    (where RMSF.py:39 raises ZeroDivisionError) is skipped, and a run with no
    frame at all raises ZeroDivisionError."""
    if order not in MERGE_ORDERS:
        raise ValueError(f"order must be one of {MERGE_ORDERS}")
    if sum(S[0] for S in parts) == 0:
        raise ZeroDivisionError("no frames on any rank")
    parts = [_empty_as_zeros(S) for S in parts]
    return (mpi4py_reduce if order == "mpi4py" else naive_reduce)(parts, _op_or_skip)


# ---------------------------------------------------------------------------
# the per-rank loops


def centred_reference(pos_sel, masses=None):
    """RMSF.py:84-85 / 117-118: (ref_com, ref_coordinates) in float64."""
    ref_com = center_of_mass(pos_sel, masses).astype(np.float64)
    ref_coordinates = pos_sel.astype(np.float64) - ref_com
    return ref_com, ref_coordinates


def align_frame_(positions: np.ndarray, masses, ref_coordinates, ref_com) -> np.ndarray:
    """RMSF.py:94-101 on the selection rows (every atom is transformed
    independently, so restricting to the selection is exact).
    ``positions`` is float32 and is modified in place, as ts.positions is."""
    mobile_com = center_of_mass(positions, masses).astype(np.float64)
    mobile_coordinates = positions.astype(np.float64) - mobile_com
    reshaped_matrix = get_rotation_matrix(ref_coordinates, mobile_coordinates, len(positions))
    return apply_transform_(positions, reshaped_matrix, mobile_com, ref_com)


def apply_transform_(positions: np.ndarray, R: np.ndarray, mobile_com, ref_com) -> np.ndarray:
    """RMSF.py:99-101 (= 133-135) with a given rotation (3x3, row-major) and
    mobile centre of mass: float32 ``positions`` rewritten in place, rounded
    to float32 after each of the three steps as ts.positions is."""
    positions[:] -= mobile_com
    positions[:] = np.dot(positions, R)
    positions += ref_com
    return positions


def rank_sweep1(traj, sel, masses, start, stop, ref_coordinates, ref_com):
    """RMSF.py:89-105 (selection rows): f64 sum of aligned float32 positions."""
    pos = np.zeros((len(sel), 3))
    for frame in range(start, stop):
        p = traj[frame][sel].astype(np.float32, copy=True)
        align_frame_(p, masses, ref_coordinates, ref_com)
        pos += p
    return pos


def rank_sweep2(traj, sel, masses, start, stop, ref_coordinates=None, ref_com=None):
    """RMSF.py:120-140: Welford on the (optionally aligned) selection.
    Returns S = [n_local, mean, sumsquares]."""
    sumsquares = np.zeros((len(sel), 3))
    mean = sumsquares.copy()
    for k, frame in enumerate(range(start, stop)):
        p = traj[frame][sel].astype(np.float32, copy=True)
        if ref_coordinates is not None:
            align_frame_(p, masses, ref_coordinates, ref_com)
        x = p.astype(np.float64)
        sumsquares += (k / (k + 1.0)) * (x - mean) ** 2
        mean = (k * mean + x) / (k + 1)
    return [stop - start, mean, sumsquares]


def _frame_list(n_traj, start, stop, step):
    return list(range(n_traj)[slice(start, stop, step)])


def rmsf_script(traj, sel=None, masses=None, size: int = 1, ref_frame: int = 0, align: str | None = "average",
                start=None, stop=None, step=None, average_f32: bool = False, merge_order: str = "mpi4py"):
    """RMSF.py end to end, emulating ``mpirun -n size`` by running the ranks
    one after another.  align="average" is the script itself; "frame0" skips
    sweep 1 and aligns on frame ``ref_frame``; None is the bare Welford.
    ``average_f32``: RMSF.py:113's MemoryReader taken to store the average
    as float32 (the other reading of an unpinned upstream detail; default
    f64, the build's choice) before the pass-2 reference of :116-118.

    Returns dict(rmsf, mean, m2, n, parts, average)."""
    traj = np.asarray(traj)
    sel = np.arange(traj.shape[1]) if sel is None else np.asarray(sel)
    fl = _frame_list(traj.shape[0], start, stop, step)
    sub = traj[fl] if (start, stop, step) != (None, None, None) else traj
    n_frames = len(fl)
    blocks = block_ranges(n_frames, size)
    average = None
    ref_coordinates = ref_com = None
    if align is not None:
        ref_com, ref_coordinates = centred_reference(traj[ref_frame][sel], masses)
    if align == "average":
        total = np.zeros((len(sel), 3))
        for b in blocks:  # Allreduce(SUM) of the per-rank sums
            total += rank_sweep1(sub, sel, masses, b.start, b.stop, ref_coordinates, ref_com)
        positions = total.reshape(-1) / float(n_frames)
        average = positions.reshape(-1, 3)
        ref_com, ref_coordinates = centred_reference(average.astype(np.float32) if average_f32 else average, masses)
    parts = [rank_sweep2(sub, sel, masses, b.start, b.stop, ref_coordinates, ref_com) for b in blocks]
    Data = chan_fold(parts, merge_order)  # RMSF.py:143
    RMSF = np.sqrt(Data[2].sum(axis=1) / Data[0])
    return dict(rmsf=RMSF, mean=Data[1], m2=Data[2], n=Data[0], parts=parts, average=average)


def rmsf_two_pass(traj, sel=None):
    """Independent check of the no-alignment statistics: two-pass variance."""
    x = np.asarray(traj, dtype=np.float64)
    if sel is not None:
        x = x[:, sel]
    mu = x.mean(axis=0)
    m2 = ((x - mu) ** 2).sum(axis=0)
    return np.sqrt(m2.sum(axis=1) / x.shape[0])


def kabsch(ref_centred, mob_centred):
    """Independent SVD superposition: R such that mob @ R ~ ref."""
    H = mob_centred.T @ ref_centred
    U, _, Vt = np.linalg.svd(H)
    d = np.sign(np.linalg.det(U @ Vt))
    D = np.diag([1.0, 1.0, d])
    return U @ D @ Vt
