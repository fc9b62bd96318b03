"""Parity against vectors produced by executing the reference's own statements.

``tests/golden/reference_exec.npz`` was written by
``tests/golden/make_reference_vectors.py``, which runs RMSF.py's own lines
(36-41 ``second_order_moments``, 43-51 ``get_rotation_matrix``, 66-69 frame
blocks, 85/95/97/99-103/105/111/118/128/131/133-138/140/146) on seeded
synthetic frames, with only the absent dependencies supplied from outside
(frames + selection, the upstream COM formula, the KAT-pinned QCP; see that
script).  CPU tier: the oracle and the C-ABI host entry points reproduce the
reference bit for bit.  GPU tier: the HIP path is within the north star's
1e-6 A of the reference.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import rmsf_oracle as O
from oracle import synth as SY

TOL = 1e-6  # Angstrom, absolute (north star)


@pytest.fixture(scope="module")
def ref():
    return np.load(os.path.join(GOLDEN, "reference_exec.npz"))


@pytest.fixture(scope="module")
def traj(ref):
    return SY.frames(int(ref["seed"]), int(ref["n_atoms"]), 0, int(ref["n_frames"]), ref["motion"])


# -- CPU tier ------------------------------------------------------------------

def test_blocks_match_reference_lines_66_69(ref):
    from rmsf_amd.engine import block_range
    for n, p, r, s, e in ref["blocks"]:
        b = O.block_ranges(int(n), int(p))[int(r)]
        assert (b.start, b.stop) == (s, e)
        assert block_range(int(n), int(p), int(r)) == (s, e)  # C ABI rmsf_block_range


def test_chan_matches_reference_lines_36_41(ref):
    for i in range(len(ref["chan_n1"])):
        S1 = (int(ref["chan_n1"][i]), ref["chan_mu1"][i], ref["chan_M1"][i])
        S2 = (int(ref["chan_n2"][i]), ref["chan_mu2"][i], ref["chan_M2"][i])
        T, mu, M = O.second_order_moments(S1, S2)
        assert T == ref["chan_T"][i]
        np.testing.assert_array_equal(mu, ref["chan_mu"][i])
        np.testing.assert_array_equal(M, ref["chan_M"][i])


@pytest.mark.parametrize("tag", ["ca", "het"])
@pytest.mark.parametrize("P", [1, 2, 3])
def test_oracle_bitwise_vs_reference(ref, traj, tag, P):
    """The numpy restatement (selection rows only) equals the reference's own
    statements (all atoms transformed) bit for bit."""
    r = O.rmsf_script(traj, ref["sel"], ref[f"masses_{tag}"], size=P, align="average")
    np.testing.assert_array_equal(r["rmsf"], ref[f"rmsf_{tag}_P{P}"])
    if P == 1:
        np.testing.assert_array_equal(r["mean"], ref[f"mean_{tag}"])
        np.testing.assert_array_equal(r["m2"], ref[f"m2_{tag}"])
        np.testing.assert_array_equal(r["average"], ref[f"average_{tag}"])


@pytest.mark.parametrize("tag", ["ca", "het"])
@pytest.mark.parametrize("P", [1, 2, 3])
def test_oracle_bitwise_vs_reference_avg32(ref, traj, tag, P):
    """The other reading of RMSF.py:113 (MemoryReader storing float32): the
    restatement's ``average_f32`` equals the reference statements run that
    way, bit for bit."""
    r = O.rmsf_script(traj, ref["sel"], ref[f"masses_{tag}"], size=P, align="average", average_f32=True)
    np.testing.assert_array_equal(r["rmsf"], ref[f"rmsf_{tag}_P{P}_avg32"])
    if P == 1:
        np.testing.assert_array_equal(r["mean"], ref[f"mean_{tag}_avg32"])


def test_memoryreader_readings_gap(ref):
    """RMSF.py:113's two readings (f64 / float32 MemoryReader) stay inside the
    north star's 1e-6 A of each other: C1 shape (both mass sets, all P) and
    100k atoms x 256 frames (max over all atoms, recorded at generation)."""
    gaps = {}
    for tag in ("ca", "het"):
        for P in (1, 2, 3):
            gaps[tag, P] = np.abs(ref[f"rmsf_{tag}_P{P}"] - ref[f"rmsf_{tag}_P{P}_avg32"]).max()
    print(f"\nC1 shape |f64 - f32 reading| max: {max(gaps.values()):.3e} A; "
          f"100k x 256: max {float(ref['big_gap_max']):.3e} mean {float(ref['big_gap_mean']):.3e} A")
    assert max(gaps.values()) < 0.5 * TOL
    assert float(ref["big_gap_max"]) < 0.5 * TOL
    assert np.abs(ref["big_rmsf"] - ref["big_rmsf_avg32"]).max() <= float(ref["big_gap_max"])


def test_oracle_100k_rows_vs_reference(ref):
    """At 100k x 256 the restatement's rows equal the reference statements'
    (both readings; every atom selected, so the reference's all-atom
    transform and the restatement's coincide)."""
    n, nf = int(ref["big_n_atoms"]), int(ref["big_n_frames"])
    t = SY.frames(int(ref["big_seed"]), n, 0, nf, ref["big_motion"])
    m = np.full(n, 12.011)
    rows = ref["big_rows"]
    r64 = O.rmsf_script(t, None, m, size=1, align="average")
    np.testing.assert_array_equal(r64["rmsf"][rows], ref["big_rmsf"])
    r32 = O.rmsf_script(t, None, m, size=1, align="average", average_f32=True)
    np.testing.assert_array_equal(r32["rmsf"][rows], ref["big_rmsf_avg32"])


def test_uniform_default_vs_ca_masses(ref, traj):
    """masses=None (centroid) vs the reference's CA masses: COM rounding moves
    a few f32 rounding points, far inside the tolerance."""
    r = O.rmsf_script(traj, ref["sel"], None, size=1, align="average")
    assert np.abs(r["rmsf"] - ref["rmsf_ca_P1"]).max() < 1e-7


@pytest.fixture(scope="module")
def lit():
    return np.load(os.path.join(GOLDEN, "reference_literal.npz"))


@pytest.fixture(scope="module")
def lit_traj(lit):
    return SY.frames(int(lit["seed"]), int(lit["n_atoms"]), 0, int(lit["frames"].max()), lit["motion"])


def test_oracle_bitwise_vs_reference_literal_shape(lit, lit_traj):
    """RMSF.py's own input shape (47,681 atoms, 214 CA, 10 frames, P = 1 and
    2 as ``mpirun -n 2``) and the same at 2 and 4 frames: the restatement
    equals the reference statements bit for bit (rmsf, mean, sumsquares and
    the sweep-1 average)."""
    for nf in lit["frames"]:
        for P in lit["sizes"]:
            r = O.rmsf_script(lit_traj[:nf], lit["sel"], lit["masses"], size=int(P), align="average")
            for k in ("rmsf", "mean", "m2", "average"):
                np.testing.assert_array_equal(r[k], lit[f"{k}_F{nf}_P{P}"], err_msg=f"{k}, {nf} frames, P={P}")
            assert [[b.start, b.stop] for b in O.block_ranges(int(nf), int(P))] == lit[f"blocks_F{nf}_P{P}"].tolist()


# -- GPU tier ------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["ca", "het"])
@pytest.mark.parametrize("where", ["device", "host"])
def test_hip_rmsf_vs_reference(ref, traj, tag, where):
    import torch

    from rmsf_amd import RMSF
    x = torch.tensor(traj, device="cuda") if where == "device" else traj
    r = RMSF(x, select=ref["sel"], align="average", masses=ref[f"masses_{tag}"]).run()
    np.testing.assert_allclose(r.results.rmsf, ref[f"rmsf_{tag}_P1"], rtol=0, atol=TOL)
    # the average structure: a rare f32 rounding flip (different COM/QCP
    # summation order) moves one coordinate by ulp/n_frames (3.9e-8 A seen)
    np.testing.assert_allclose(r.results.average, ref[f"average_{tag}"], rtol=0, atol=TOL)
    assert r.results.n_frames == int(ref["n_frames"])
    # the other reading of RMSF.py:113 (float32 MemoryReader)
    np.testing.assert_allclose(r.results.rmsf, ref[f"rmsf_{tag}_P1_avg32"], rtol=0, atol=TOL)
    # default (uniform masses) against the reference's CA masses
    r = RMSF(x, select=ref["sel"], align="average").run()
    np.testing.assert_allclose(r.results.rmsf, ref["rmsf_ca_P1"], rtol=0, atol=TOL)


@pytest.mark.gpu
def test_hip_rmsf_100k_vs_both_readings(ref):
    """100k atoms x 256 frames, RMSF.py's two sweeps on the device: the
    sampled rows within 1e-6 A of the reference statements under both
    readings of RMSF.py:113."""
    import torch

    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    n, nf = int(ref["big_n_atoms"]), int(ref["big_n_frames"])
    t = generate(Engine(), n, 0, nf, seed=int(ref["big_seed"]), motion=ref["big_motion"])
    r = RMSF(t, align="average", masses=np.full(n, 12.011)).run().results
    rows = ref["big_rows"]
    d64 = np.abs(r.rmsf[rows] - ref["big_rmsf"]).max()
    d32 = np.abs(r.rmsf[rows] - ref["big_rmsf_avg32"]).max()
    print(f"\n100k x 256: build vs f64 reading {d64:.3e} A, vs f32 reading {d32:.3e} A")
    assert d64 < TOL and d32 < TOL
    np.testing.assert_allclose(r.average[rows], ref["big_average"], rtol=0, atol=TOL)
    del t
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_hip_chan_merge_vs_reference(ref):
    from rmsf_amd import second_order_moments
    for i in range(len(ref["chan_n1"])):
        S1 = (int(ref["chan_n1"][i]), ref["chan_mu1"][i], ref["chan_M1"][i])
        S2 = (int(ref["chan_n2"][i]), ref["chan_mu2"][i], ref["chan_M2"][i])
        T, mu, M = second_order_moments(S1, S2)
        assert T == ref["chan_T"][i]
        # bit for bit: k_chan_merge writes RMSF.py:36-41's expressions in
        # numpy's order and the library is built without FP contraction
        np.testing.assert_array_equal(np.asarray(mu).view(np.uint64), np.asarray(ref["chan_mu"][i]).view(np.uint64))
        np.testing.assert_array_equal(np.asarray(M).view(np.uint64), np.asarray(ref["chan_M"][i]).view(np.uint64))
