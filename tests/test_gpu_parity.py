"""GPU tier, end to end: ``RMSF(...).run().results.rmsf`` on the HIP path vs the
oracle restatement of RMSF.py, within the north star's 1e-6 A (absolute).

Covers the three modes (None / frame0 / average = RMSF.py), device-resident
and host-streamed (pinned stager) inputs, gathered selections, masses, frame
slicing, split/batch invariance, edge cases, and -- at the full 100k-atom
size -- slice checks regenerated on the CPU."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6  # Angstrom, absolute (north star)


@pytest.fixture(scope="module")
def c1():
    d = np.load(os.path.join(GOLDEN, "c1_synth.npz"))
    traj = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, int(d["n_frames"]), d["motion"])
    return d, traj


@pytest.mark.parametrize("align,tag", [(None, "none"), ("frame0", "frame0"), ("average", "average")])
@pytest.mark.parametrize("where", ["device", "host"])
def test_c1_modes_vs_golden(c1, align, tag, where):
    from rmsf_amd import RMSF
    d, traj = c1
    x = torch.tensor(traj, device="cuda") if where == "device" else traj
    r = RMSF(x, select=d["sel"], align=align).run()
    np.testing.assert_allclose(r.results.rmsf, d[f"rmsf_{tag}_P1"], rtol=0, atol=TOL)
    np.testing.assert_allclose(r.results.mean, d[f"mean_{tag}"], rtol=0, atol=1e-6)
    assert r.results.n_frames == 98
    if align == "average":
        np.testing.assert_allclose(r.results.average, d["average"], rtol=0, atol=1e-9)


def test_c1_masses_and_slices(c1):
    from rmsf_amd import RMSF
    d, traj = c1
    x = torch.tensor(traj, device="cuda")
    r = RMSF(x, select=d["sel"], align="average", masses=d["masses"]).run()
    np.testing.assert_allclose(r.results.rmsf, d["rmsf_average_masses_P2"], atol=TOL)
    r = RMSF(x, select=d["sel"], align="average").run(start=3, stop=90, step=2)
    np.testing.assert_allclose(r.results.rmsf, d["rmsf_average_slice"], atol=TOL)
    r = RMSF(traj, select=d["sel"], align="average", batch_frames=7).run(start=3, stop=90, step=2)
    np.testing.assert_allclose(r.results.rmsf, d["rmsf_average_slice"], atol=TOL)


@pytest.mark.parametrize("batch,splits", [(1, 1), (5, 2), (13, None), (98, 3)])
def test_batch_and_split_invariance(c1, batch, splits):
    """Frame tiles inside a GPU (splits) and streamed batches are merged by the
    same Chan kernel as ranks are; any cut gives the same answer."""
    from rmsf_amd import RMSF
    d, traj = c1
    x = torch.tensor(traj, device="cuda")
    r = RMSF(x, select=d["sel"], align="average", batch_frames=batch, n_splits=splits).run()
    np.testing.assert_allclose(r.results.rmsf, d["rmsf_average_P1"], atol=TOL)


def test_edges():
    from rmsf_amd import RMSF, RmsfEmptyError
    d = np.load(os.path.join(GOLDEN, "edges.npz"))
    t3 = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, 3, d["motion"])
    one = RMSF(torch.tensor(t3[:1], device="cuda"), align="average").run()
    np.testing.assert_array_equal(one.results.rmsf, 0.0)  # RMSF of one frame is exactly 0
    ident = RMSF(np.repeat(t3[:1], 10, axis=0), align="average").run()
    assert ident.results.rmsf.max() < 1e-6
    r = RMSF(torch.tensor(t3, device="cuda"), align="average").run()
    np.testing.assert_allclose(r.results.rmsf, d["p1_of_3"], atol=TOL)
    with pytest.raises(ZeroDivisionError):
        RMSF(torch.tensor(t3, device="cuda")).run(start=2, stop=2)
    assert issubclass(RmsfEmptyError, ZeroDivisionError)


def test_one_atom_superposition_nan_like_qcprot():
    """RMSF.py with a one-atom selection: the superposition is undefined --
    qcprot's Newton step divides 0 by 0, the rotation is NaN and so is the
    RMSF (the oracle, restating qcprot, gives NaN).  The device propagates
    the NaN whatever the frame count and batching (M2's clamp at 0 is a
    comparison, not fmax, which turned NaN into 0 for some segment splits)."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    traj = SY.frames(5, 191, 0, 11, motion_table(7, 11))
    planes = torch.tensor(np.ascontiguousarray(traj.transpose(0, 2, 1)), device="cuda")
    for frames in (np.array([0, 2, 5, 9]), np.arange(11)):
        exp = O.rmsf_script(traj[frames], np.array([40]), None, size=1, align="frame0")["rmsf"]
        assert np.isnan(exp).all()
        for x, kw in ((traj, {}), (torch.tensor(traj, device="cuda"), {}), (planes, {"layout": "soa"})):
            for bf in (None, 3):
                r = RMSF(x, select=[40], align="frame0", batch_frames=bf, **kw).run(frames=frames)
                assert np.isnan(r.results.rmsf).all(), (kw, bf, r.results.rmsf)
    # without alignment one atom is well defined
    r = RMSF(traj, select=[40]).run()
    exp = O.rmsf_script(traj, np.array([40]), None, size=1, align=None)["rmsf"]
    np.testing.assert_allclose(r.results.rmsf, exp, atol=TOL)


def test_rigid_motion_removed():
    """Analytic: rigid copies of one structure -> RMSF at the f32 floor."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    one = SY.frames(40, 3000, 0, 1)[0].astype(np.float64) - 50.0
    mt = motion_table(41, 64)
    traj = np.stack([(one @ mt[f, :9].reshape(3, 3) + mt[f, 9:]).astype(np.float32) for f in range(64)])
    r = RMSF(torch.tensor(traj, device="cuda"), align="frame0").run()
    assert r.results.rmsf.max() < 2e-5
    exp = O.rmsf_script(traj, None, align="frame0")["rmsf"]
    np.testing.assert_allclose(r.results.rmsf, exp, atol=TOL)


def test_rmsd_byproduct(c1):
    from rmsf_amd import RMSF
    d, traj = c1
    r = RMSF(torch.tensor(traj, device="cuda"), select=d["sel"], align="frame0", collect_rmsd=True).run()
    sel = d["sel"]
    ref_com, ref_c = O.centred_reference(traj[0][sel])
    exp = []
    for f in range(len(traj)):
        p = traj[f][sel]
        A, E0 = O.inner_product(ref_c, p.astype(np.float64) - O.center_of_mass(p))
        exp.append(O.fast_calc_rmsd_and_rotation(A, E0, float(len(sel)))[1])
    # rmsd = sqrt(|2 (E0 - lambda) / N|): near 0 (frame 0 is the reference)
    # the square root turns the rounding of E0 - lambda (~1e-12 A^2, any
    # summation order) into ~1e-6 A, so compare the squares
    exp = np.array(exp)
    np.testing.assert_allclose(r.results.rmsd ** 2, exp ** 2, rtol=0, atol=1e-8)
    np.testing.assert_allclose(r.results.rmsd[1:], exp[1:], rtol=0, atol=1e-7)


def test_full_size_noalign_slices():
    """C2 shape (100k atoms) at 2k frames: full-width result, CPU-verified on
    sampled atoms regenerated bit-exactly from the counter-based generator."""
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    eng = Engine()
    n_atoms, nf = 100_000, 2000
    traj = generate(eng, n_atoms, 0, nf, seed=0)
    r = RMSF(traj).run()
    atoms = np.random.default_rng(0).choice(n_atoms, 64, replace=False)
    host = SY.frames(0, n_atoms, 0, nf, atoms=atoms)
    np.testing.assert_allclose(r.results.rmsf[atoms], O.rmsf_two_pass(host), atol=1e-9)
    # size-independent property: close to the analytic sqrt(3) sigma
    np.testing.assert_allclose(r.results.rmsf, SY.expected_rmsf(0, np.arange(n_atoms)), rtol=0.12)
    del traj


def test_full_size_aligned_slices():
    """C3 shape (100k atoms, QCP to frame 0) at 256 frames; the per-atom
    result of sampled atoms is rebuilt on the CPU from the GPU's own frames."""
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    eng = Engine()
    n_atoms, nf = 100_000, 256
    mt = motion_table(1, nf)
    traj = generate(eng, n_atoms, 0, nf, seed=0, motion=mt)
    r = RMSF(traj, align="frame0").run()
    host = traj.cpu().numpy()
    exp = O.rmsf_script(host, None, align="frame0")["rmsf"]
    np.testing.assert_allclose(r.results.rmsf, exp, atol=TOL)


def test_bitwise_reproducible(c1):
    """Fixed-order reductions, no atomics: two runs agree bit for bit."""
    from rmsf_amd import RMSF
    d, traj = c1
    x = torch.tensor(traj, device="cuda")
    a = RMSF(x, select=d["sel"], align="average").run().results
    b = RMSF(x, select=d["sel"], align="average").run().results
    np.testing.assert_array_equal(a.rmsf, b.rmsf)
    np.testing.assert_array_equal(a.sumsquares, b.sumsquares)
    np.testing.assert_array_equal(a.average, b.average)


def test_captured_pipeline_replay(c1):
    """hipGraph replay == eager run bit for bit, and tracks in-place input
    updates (frames rewritten between replays)."""
    from rmsf_amd.engine import Engine
    from rmsf_amd.pipeline import CapturedPipeline, run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList
    d, traj = c1
    eng = Engine()
    x = torch.tensor(traj, device="cuda")
    src, fl = DeviceSource(x, d["sel"]), FrameList(len(traj))
    cap = CapturedPipeline(eng, src, fl, align="average")
    eager = run_pipeline(eng, src, fl, align="average")
    r = cap.replay()
    torch.cuda.synchronize()
    assert torch.equal(r.rmsf, eager.rmsf) and torch.equal(r.average, eager.average)
    np.testing.assert_allclose(r.rmsf.cpu().numpy(), d["rmsf_average_P1"], atol=TOL)
    x.copy_(torch.flip(x, dims=[0]))  # new data, same buffer
    r = cap.replay()
    torch.cuda.synchronize()
    exp = O.rmsf_script(traj[::-1].copy(), d["sel"], None, size=1, align="average")["rmsf"]
    np.testing.assert_allclose(r.rmsf.cpu().numpy(), exp, atol=TOL)


@pytest.mark.parametrize("kw", [{}, dict(start=3, stop=90, step=2)])
def test_host_frame_cache(c1, kw):
    """RMSF.py's second loop (RMSF.py:124) reads the frames the first staged:
    with the HBM frame cache the two sweeps of a host array cross PCIe once,
    bit-identical to streaming them twice."""
    from rmsf_amd import RMSF
    from rmsf_amd.sources import HostSource
    d, traj = c1
    plain = RMSF(HostSource(traj, d["sel"], batch_frames=7), align="average").run(**kw).results
    src = HostSource(traj, d["sel"], batch_frames=7, cache=True)
    got = RMSF(src, align="average").run(**kw).results
    assert src.cache is not None
    used = np.arange(98)[slice(kw.get("start"), kw.get("stop"), kw.get("step"))]
    assert src.cache.have[used].all()
    np.testing.assert_array_equal(got.rmsf, plain.rmsf)
    np.testing.assert_array_equal(got.average, plain.average)
    np.testing.assert_allclose(got.rmsf, d["rmsf_average_P1" if not kw else "rmsf_average_slice"], rtol=0, atol=TOL)


@pytest.mark.parametrize("align", [None, "frame0", "average"])
@pytest.mark.parametrize("where", ["device", "host"])
def test_explicit_frames(c1, align, where):
    """run(frames=...) (MDAnalysis AnalysisBase): indices with gaps, strided
    stretches and a repeated frame, or the same selection as a boolean mask,
    equal RMSF over the trajectory of just those frames.  Frame 0 is
    selected, so the frame-0 reference (RMSF.py:80-87) is the same frame."""
    from rmsf_amd import RMSF
    d, traj = c1
    idx = np.array([0, 3, 4, 5, 9, 15, 21, 27, 33, 34, 34, 60, 61, 62, 63, 97])
    x = torch.tensor(traj, device="cuda") if where == "device" else traj
    got = RMSF(x, select=d["sel"], align=align, batch_frames=5).run(frames=idx).results
    exp = RMSF(traj[idx], select=d["sel"], align=align).run().results
    assert got.n_frames == len(idx)
    np.testing.assert_allclose(got.rmsf, exp.rmsf, rtol=0, atol=1e-9)
    mask = np.zeros(98, bool)
    mask[idx] = True
    got = RMSF(x, select=d["sel"], align=align).run(frames=mask).results
    exp = RMSF(traj[mask], select=d["sel"], align=align).run().results
    np.testing.assert_allclose(got.rmsf, exp.rmsf, rtol=0, atol=1e-9)
    ref = O.rmsf_script(traj[mask], d["sel"], None, size=1, align=align)["rmsf"]
    np.testing.assert_allclose(got.rmsf, ref, rtol=0, atol=TOL)


@pytest.mark.parametrize("align", [None, "average"])
@pytest.mark.parametrize("where", ["device", "host", "host_cache", "dcd", "atomgroup"])
def test_scattered_frames_gathered_batches(tmp_path, c1, align, where):
    """A scattered frame list (runs of 1-2 frames) is read as compact gathered
    batches -- rmsf_gather_frames from HBM (and from the HBM frame cache on the
    second sweep), pointer-staged host rows, per-run DCD reads, per-frame
    AtomGroup positions -- one set of launches per batch instead of per run;
    equal to the oracle on just those frames."""
    from rmsf_amd import RMSF
    from rmsf_amd.sources import AtomGroupSource, DcdSource, HostSource
    from test_gpu_multirank import _FakeAtomGroup, _FakeUniverse
    d, traj = c1
    sel = d["sel"]
    idx = np.sort(np.random.default_rng(5).choice(np.arange(1, 98), 40, replace=False))
    idx = np.concatenate([[0], idx])  # frame 0 in the list: the frame-0 reference is the list's first frame
    if where == "device":
        src = torch.tensor(traj, device="cuda")
    elif where == "host":
        src = HostSource(traj, sel, batch_frames=9)
    elif where == "host_cache":
        src = HostSource(traj, sel, batch_frames=9, cache=True)
    elif where == "dcd":
        from rmsf_amd.dcd import write_dcd
        p = str(tmp_path / "t.dcd")
        write_dcd(p, traj)
        src = DcdSource(p, sel, batch_frames=9, cache=align == "average")
    else:
        src = AtomGroupSource(_FakeAtomGroup(_FakeUniverse(traj), sel, np.ones(len(sel))), batch_frames=9,
                              cache=align == "average")
    kw = dict(select=sel) if where == "device" else {}
    got = RMSF(src, align=align, batch_frames=9, **kw).run(frames=idx).results
    exp = O.rmsf_script(traj[idx], sel, None, size=1, align=align)["rmsf"]
    assert got.n_frames == len(idx)
    np.testing.assert_allclose(got.rmsf, exp, rtol=0, atol=TOL)
    if where == "host_cache" and align == "average":
        assert src.cache.have[idx].all() and src.cache.have.sum() == len(idx)
