"""CPU tier: the oracle pinned against known answers, independent methods and
the committed golden vectors (no GPU needed)."""
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import GOLDEN
from oracle import rmsf_oracle as O
from oracle import synth as SY


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


# -- QCP ---------------------------------------------------------------------

def test_qcp_known_answer_upstream():
    """upstream MDAnalysisTests test_qcprot.py vector."""
    d = _load("qcp_kat.npz")
    ref = d["ref"] - d["ref"].mean(axis=0)
    mob = d["mob"] - d["mob"].mean(axis=0)
    rot = np.zeros(9)
    rmsd = O.CalcRMSDRotationalMatrix(ref, mob, 7, rot, None)
    assert rmsd == pytest.approx(float(d["rmsd"]), abs=1e-6)
    assert rmsd == pytest.approx(0.7191064509622, abs=1e-12)
    np.testing.assert_allclose(rot.reshape(3, 3), d["rot"], atol=1e-7)
    # applied as mob @ R it superposes onto ref
    fit = np.sqrt(((mob @ rot.reshape(3, 3) - ref) ** 2).sum() / 7)
    assert fit == pytest.approx(rmsd, abs=1e-9)


def _inner_product_loop(ref, conf, w=None):
    """qcprot's InnerProduct as its published C loop (one pass, per-atom
    updates, no contraction) in plain Python floats (upstream, unverified)."""
    A = [0.0] * 9
    G1 = G2 = 0.0
    for i in range(len(conf)):
        wi = 1.0 if w is None else float(w[i])
        c = [float(v) for v in conf[i]]
        x1, y1, z1 = (c if w is None else [wi * v for v in c])
        G1 += x1 * c[0] + y1 * c[1] + z1 * c[2]
        x2, y2, z2 = (float(v) for v in ref[i])
        G2 += (x2 * x2 + y2 * y2 + z2 * z2) if w is None else wi * (x2 * x2 + y2 * y2 + z2 * z2)
        for a, p in enumerate((x1, y1, z1)):
            for b, r in enumerate((x2, y2, z2)):
                A[3 * a + b] += p * r
    return A, (G1 + G2) * 0.5


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("n", [1, 7, 214, 1500])
def test_inner_product_follows_qcprot_loop(n, weighted):
    """The oracle's vectorised InnerProduct sums in the published loop's
    order: A, G1, G2 and E0 equal the per-atom loop bit for bit (item 3 of
    the round-5 verdict: E0 no longer summed pairwise)."""
    rng = np.random.default_rng(n)
    ref = rng.normal(size=(n, 3)) * 20
    conf = rng.normal(size=(n, 3)) * 20
    w = rng.uniform(1, 16, n) if weighted else None
    A, E0 = O.inner_product(ref, conf, w)
    A2, E02 = _inner_product_loop(ref, conf, w)
    assert A == A2
    assert E0 == E02


@pytest.mark.parametrize("seed", range(20))
def test_qcp_matches_kabsch(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(3, 300))
    ref = rng.normal(size=(n, 3)) * 10
    R0 = O.kabsch(rng.normal(size=(3, 3)), rng.normal(size=(3, 3)))
    mob = ref @ R0.T + rng.normal(size=(n, 3)) * rng.uniform(0, 2)
    ref -= ref.mean(0)
    mob -= mob.mean(0)
    R = O.get_rotation_matrix(ref, mob, n)
    np.testing.assert_allclose(R, O.kabsch(ref, mob), atol=1e-8)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
    assert np.linalg.det(R) == pytest.approx(1.0, abs=1e-12)


def test_qcp_identity_and_degenerate():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(50, 3))
    x -= x.mean(0)
    R = O.get_rotation_matrix(x, x, 50)
    np.testing.assert_allclose(R, np.eye(3), atol=1e-8)
    # all-zero input (e.g. a 1-atom selection): Newton divides 0/0 and the C
    # algorithm propagates NaN -- the oracle keeps C's IEEE semantics
    z = np.zeros((5, 3))
    rot, rmsd, _ = O.fast_calc_rmsd_and_rotation(O.inner_product(z, z)[0], 0.0, 5.0)
    assert all(np.isnan(rot)) and np.isnan(rmsd)


def test_qcp_adjugate_fallback_columns():
    """Force the first adjugate column to vanish: a pure 180-degree rotation
    about x gives q = (0, 1, 0, 0), so column 1 (q1 from rows 3-4 minors) is
    ~0 and the later columns must still produce the right matrix."""
    rng = np.random.default_rng(3)
    ref = rng.normal(size=(40, 3))
    ref -= ref.mean(0)
    Rx = np.diag([1.0, -1.0, -1.0])
    mob = ref @ Rx.T
    R = O.get_rotation_matrix(ref, mob, 40)
    np.testing.assert_allclose(mob @ R, ref, atol=1e-8)


# -- moments -----------------------------------------------------------------

def _stats(x):
    return [len(x), x.mean(0), ((x - x.mean(0)) ** 2).sum(0)]


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(1, 40), min_size=2, max_size=6), st.integers(0, 10_000))
def test_chan_merge_equals_two_pass(sizes, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(sum(sizes), 7, 3)) * rng.uniform(0.1, 100) + rng.uniform(-1e3, 1e3)
    parts, o = [], 0
    for s in sizes:
        parts.append(_stats(x[o:o + s]))
        o += s
    n, mu, m2 = O.chan_fold(parts)
    ref = _stats(x)
    assert n == ref[0]
    np.testing.assert_allclose(mu, ref[1], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(m2, ref[2], rtol=1e-9, atol=1e-7)


def test_chan_empty_partials():
    x = np.random.default_rng(1).normal(size=(5, 4, 3))
    a = _stats(x)
    empty = [0, np.zeros((4, 3)), np.zeros((4, 3))]
    # reference semantics for one empty side: identical to the non-empty one
    n, mu, m2 = O.second_order_moments(empty, a)
    assert n == 5
    np.testing.assert_allclose(mu, a[1])
    np.testing.assert_allclose(m2, a[2])
    # two empties raise in the reference (RMSF.py:39)
    with pytest.raises(ZeroDivisionError):
        O.second_order_moments(empty, empty)
    assert O.chan_fold([empty, a, empty])[0] == 5


def test_welford_matches_two_pass():
    x = SY.frames(2, 64, 0, 200)
    S = O.rank_sweep2(x, np.arange(64), None, 0, 200)
    np.testing.assert_allclose(np.sqrt(S[2].sum(1) / S[0]), O.rmsf_two_pass(x), rtol=1e-12)


# -- blocks ------------------------------------------------------------------

@pytest.mark.parametrize("n,size", [(98, 2), (10, 3), (3, 8), (0, 4), (20000, 8), (7, 1)])
def test_block_ranges(n, size):
    b = O.block_ranges(n, size)
    assert len(b) == size
    per = n // size
    for i in range(size - 1):
        assert (b[i].start, b[i].stop) == (i * per, (i + 1) * per)
    assert (b[-1].start, b[-1].stop) == ((size - 1) * per, n)
    assert sum(len(r) for r in b) == n


# -- golden vectors ------------------------------------------------------------

def test_synth_generator_golden():
    d = _load("synth_slice.npz")
    np.testing.assert_array_equal(SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, 4), d["frames"])
    np.testing.assert_array_equal(SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, 4, d["motion"]),
                                  d["frames_motion"])
    # slices are addressable: atoms subset / later frames equal the full draw
    full = SY.frames(7, 30, 0, 6)
    np.testing.assert_array_equal(SY.frames(7, 30, 2, 3, atoms=np.arange(5, 17)), full[2:5, 5:17])


def test_synth_statistics():
    """Unaligned generator: RMSF -> sqrt(3) sigma (analytic)."""
    x = SY.frames(4, 200, 0, 3000)
    got = O.rmsf_two_pass(x)
    np.testing.assert_allclose(got, SY.expected_rmsf(4, np.arange(200)), rtol=0.05)


def _c1_traj():
    d = _load("c1_synth.npz")
    traj = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, int(d["n_frames"]), d["motion"])
    return d, traj


def test_oracle_c1_golden():
    d, traj = _c1_traj()
    sel = d["sel"]
    for align, tag in ((None, "none"), ("frame0", "frame0"), ("average", "average")):
        for P in (1, 2, 8):
            r = O.rmsf_script(traj, sel, None, size=P, align=align)
            np.testing.assert_allclose(r["rmsf"], d[f"rmsf_{tag}_P{P}"], rtol=0, atol=1e-12)
    r = O.rmsf_script(traj, sel, d["masses"], size=2, align="average")
    np.testing.assert_allclose(r["rmsf"], d["rmsf_average_masses_P2"], rtol=0, atol=1e-12)


def test_oracle_block_invariance():
    d, traj = _c1_traj()
    for tag in ("none", "frame0", "average"):
        np.testing.assert_allclose(d[f"rmsf_{tag}_P1"], d[f"rmsf_{tag}_P2"], atol=1e-12)
        np.testing.assert_allclose(d[f"rmsf_{tag}_P1"], d[f"rmsf_{tag}_P8"], atol=1e-12)


def test_alignment_removes_rigid_motion():
    """Analytic: frames that differ only by rigid motions have RMSF ~ 0 after
    superposition (f32 rounding floor), and huge RMSF without it."""
    from tests.golden.make_golden import motion_table
    one = SY.frames(40, 120, 0, 1)
    mt = motion_table(41, 30)
    p = one[0].astype(np.float64) - 50.0
    traj = np.stack([(p @ mt[f, :9].reshape(3, 3) + mt[f, 9:]).astype(np.float32) for f in range(30)])
    assert O.rmsf_script(traj, None, align=None)["rmsf"].min() > 1.0
    r = O.rmsf_script(traj, None, align="average")["rmsf"]
    assert r.max() < 2e-5


def test_oracle_noalign_golden():
    d = _load("noalign_4096.npz")
    t = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, int(d["n_frames"]))
    np.testing.assert_allclose(O.rmsf_script(t, None, size=1, align=None)["rmsf"], d["rmsf_P1"], atol=1e-12)
    np.testing.assert_allclose(O.rmsf_two_pass(t), d["rmsf_P1"], rtol=1e-10)
    np.testing.assert_allclose(d["rmsf_P3"], d["rmsf_P1"], atol=1e-12)


def test_oracle_edges_golden():
    d = _load("edges.npz")
    assert np.all(d["one_frame"] == 0.0)
    assert np.all(d["identical"] == 0.0)
    np.testing.assert_allclose(d["p8_of_3"], d["p1_of_3"], atol=1e-12)


def test_rebuild_from_transforms_equals_script():
    """The full-size GPU tests rebuild sampled atoms from per-frame (R, mobile
    COM) records: RMSF.py's loop with the records of align_frame_ must give
    rmsf_script's answer bit for bit, on a subset of rows too (every atom is
    transformed independently, RMSF.py:99-101)."""
    rng = np.random.default_rng(5)
    nf, n = 40, 30
    base = rng.normal(scale=8.0, size=(n, 3))
    traj = np.empty((nf, n, 3), dtype=np.float32)
    for f in range(nf):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        a, b, c, d = q
        R = np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                      [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                      [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])
        traj[f] = (base + rng.normal(scale=0.5, size=(n, 3))) @ R + rng.uniform(-5, 5, 3)
    exp = O.rmsf_script(traj, align="frame0")
    ref_com, ref_c = O.centred_reference(traj[0])
    T = np.zeros((nf, 16))
    for f in range(nf):
        mob = traj[f]
        com = O.center_of_mass(mob).astype(np.float64)
        T[f, :9] = O.get_rotation_matrix(ref_c, mob.astype(np.float64) - com, n).reshape(-1)
        T[f, 9:12] = com
    rows = np.array([3, 7, 8, 20, 29])
    aligned = np.empty((nf, len(rows), 3), dtype=np.float32)
    for f in range(nf):
        p = traj[f][rows].copy()
        O.apply_transform_(p, T[f, :9].reshape(3, 3), T[f, 9:12], ref_com)
        aligned[f] = p
    S = O.rank_sweep2(aligned, np.arange(len(rows)), None, 0, nf)
    np.testing.assert_array_equal(S[1], exp["mean"][rows])
    np.testing.assert_array_equal(np.sqrt(S[2].sum(axis=1) / S[0]), exp["rmsf"][rows])
