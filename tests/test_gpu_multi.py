"""GPU tier: ``RMSF(..., gpus=...)`` -- one process driving several contexts
(rmsf_amd.multi), RMSF.py:65-69 blocks per context, merged over the
in-process fold (a device listed more than once; distinct devices use RCCL
communicators, which this one-GPU box exercises in test_gpu_context.py's
ncclCommInitAll case).  Checked against the oracle's ``mpirun -n P`` emulation at the north
star's 1e-6 A, and against the one-process pipeline bit for bit where the
arithmetic is identical."""
import numpy as np
import pytest
import torch

from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def traj():
    from rmsf_amd.synth import motion_table
    return SY.frames(21, 700, 0, 37, motion_table(22, 37))


@pytest.mark.parametrize("align", [None, "frame0", "average"])
@pytest.mark.parametrize("gpus", [[0, 0, 0], [0] * 5])
def test_multi_host_array_vs_oracle(traj, align, gpus):
    from rmsf_amd import RMSF
    sel = np.arange(1, 700, 3)
    r = RMSF(traj, select=sel, align=align, gpus=gpus).run()
    exp = O.rmsf_script(traj, sel, None, size=len(gpus), align=align)
    np.testing.assert_allclose(r.results.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    np.testing.assert_allclose(r.results.mean.reshape(-1), exp["mean"].reshape(-1), rtol=0, atol=1e-9)
    assert r.results.n_frames == 37
    assert r.results.blocks == [(b.start, b.stop) for b in O.block_ranges(37, len(gpus))]
    if align == "average":
        np.testing.assert_allclose(r.results.average, exp["average"].reshape(-1), rtol=0, atol=1e-9)


def test_multi_frame_slice_masses_and_empty_blocks(traj):
    """start/stop/step, masses, and more contexts than frames (empty blocks,
    RMSF.py:65-69 with P > n)."""
    from rmsf_amd import RMSF
    sel = np.arange(0, 700, 7)
    m = np.random.default_rng(3).uniform(1, 16, len(sel))
    r = RMSF(traj, select=sel, align="average", masses=m, gpus=[0, 0]).run(start=3, stop=30, step=4)
    exp = O.rmsf_script(traj, sel, m, size=2, align="average", start=3, stop=30, step=4)
    np.testing.assert_allclose(r.results.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    r = RMSF(traj[:3], select=sel, align="frame0", gpus=[0] * 5).run()
    exp = O.rmsf_script(traj[:3], sel, None, size=5, align="frame0")
    np.testing.assert_allclose(r.results.rmsf, exp["rmsf"], rtol=0, atol=TOL)


@pytest.mark.parametrize("gpus", [1, [0]])
def test_multi_single_device_equals_pipeline(traj, gpus):
    """One device from one process (no communicator is made for a single
    context) against the pipeline on the same frames."""
    from rmsf_amd import RMSF
    sel = np.arange(2, 700, 5)
    a = RMSF(traj, select=sel, align="average", gpus=gpus).run()
    b = RMSF(torch.tensor(traj, device="cuda"), select=sel, align="average").run()
    np.testing.assert_allclose(a.results.rmsf, b.results.rmsf, rtol=0, atol=1e-12)


def test_multi_xtc(tmp_path, traj):
    from oracle import xtc_py
    from rmsf_amd import RMSF
    from rmsf_amd.xtc import write_xtc
    path = str(tmp_path / "m.xtc")
    write_xtc(path, traj)
    q = xtc_py.read_xtc(path)
    sel = np.arange(0, 700, 2)
    r = RMSF(path, select=sel, align="average", gpus=[0, 0, 0]).run(step=2)
    exp = O.rmsf_script(q, sel, None, size=3, align="average", step=2)
    np.testing.assert_allclose(r.results.rmsf, exp["rmsf"], rtol=0, atol=TOL)


def test_multi_atomgroup_duck_typed(traj):
    from rmsf_amd import RMSF
    from test_gpu_multirank import _FakeAtomGroup, _FakeUniverse
    sel = np.arange(5, 700, 9)
    m = np.random.default_rng(4).uniform(1, 16, len(sel))
    ag = _FakeAtomGroup(_FakeUniverse(traj), sel, m)
    r = RMSF(ag, align="average", gpus=[0, 0]).run()
    exp = O.rmsf_script(traj, sel, m, size=2, align="average")
    np.testing.assert_allclose(r.results.rmsf, exp["rmsf"], rtol=0, atol=TOL)


def test_multi_errors(traj):
    from rmsf_amd import RMSF
    with pytest.raises(ValueError, match="shards' devices"):
        RMSF(torch.tensor(traj, device="cuda"), gpus=[0, 0]).run()
    with pytest.raises(ZeroDivisionError):
        RMSF(traj, gpus=[0, 0]).run(start=5, stop=5)
    with pytest.raises(ValueError, match="collect_rmsd"):
        RMSF(traj, collect_rmsd=True, gpus=1).run()
    with pytest.raises(TypeError):
        RMSF([torch.tensor(traj, device="cuda").double()], gpus=1).run()


def _shards(traj, cuts):
    t = torch.tensor(traj, device="cuda")
    edges = [0] + list(cuts) + [len(traj)]
    return [t[a:b].contiguous() for a, b in zip(edges[:-1], edges[1:])]


@pytest.mark.parametrize("align", [None, "frame0", "average"])
@pytest.mark.parametrize("run", [{}, {"start": 3, "step": 4}, {"frames": [0, 1, 2, 11, 12, 30, 31, 36]},
                                 {"step": -2}])
def test_multi_device_shards(traj, align, run):
    """HBM-resident shards, one tensor per device (here: three on device 0,
    the in-process fold): each context takes the frames its shard holds;
    equal to the oracle on the same (ascending) frames."""
    from rmsf_amd import RMSF
    sel = np.arange(3, 700, 4)
    parts = _shards(traj, (10, 25))
    r = RMSF(parts, select=sel, align=align, collect_rmsd=align is not None).run(**run).results
    fl = np.sort(np.arange(len(traj))[slice(run.get("start"), None, run.get("step"))]) if "frames" not in run \
        else np.array(run["frames"])
    # the oracle on those frames, with trajectory frame 0 as the reference (RMSF.py:63,80-87)
    exp = O.rmsf_script(traj[np.concatenate([[0], fl])], sel, None, size=1, align=align, start=1)
    np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    assert r.n_frames == len(fl) and r.devices == [0, 0, 0]
    assert sum(b1 - b0 for b0, b1 in r.blocks) == len(fl)
    if align is not None:
        one = RMSF(torch.tensor(traj, device="cuda"), select=sel, align=align, collect_rmsd=True).run(frames=fl)
        np.testing.assert_allclose(r.rmsd, one.results.rmsd, rtol=0, atol=1e-9)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two visible GPUs (the cross-device branch)")
@pytest.mark.parametrize("align", ["frame0", "average"])
def test_multi_device_shards_two_devices(traj, align):
    """Shards on two distinct devices: the reference frame lives on device 0
    and is copied to device 1 (the cross-device branch of run_multi), each
    shard produced by torch's stream and read on the context stream."""
    from rmsf_amd import RMSF
    sel = np.arange(3, 700, 4)
    t = torch.tensor(traj, device="cuda:0")
    parts = [t[:20].contiguous(), t[20:].to("cuda:1")]
    r = RMSF(parts, select=sel, align=align).run().results
    exp = O.rmsf_script(traj, sel, None, size=1, align=align)
    np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    assert r.devices == [0, 1] and r.n_frames == len(traj)


@pytest.mark.parametrize("align", ["frame0", "average"])
def test_multi_collect_rmsd_host(traj, align):
    """The per-frame QCP rmsd (RMSF.py:48's discarded by-product) under gpus=,
    in frame-list order across the devices' blocks."""
    from rmsf_amd import RMSF
    sel = np.arange(0, 700, 5)
    r = RMSF(traj, select=sel, align=align, collect_rmsd=True, gpus=[0, 0, 0]).run(step=2).results
    one = RMSF(torch.tensor(traj, device="cuda"), select=sel, align=align, collect_rmsd=True).run(step=2).results
    assert r.rmsd.shape == (len(range(0, len(traj), 2)),)
    np.testing.assert_allclose(r.rmsd, one.rmsd, rtol=0, atol=1e-9)


@pytest.mark.parametrize("sl", [dict(step=-2), dict(start=30, stop=2, step=-3)])
def test_multi_reversed_ranges(traj, sl):
    from rmsf_amd import RMSF
    sel = np.arange(1, 700, 6)
    r = RMSF(traj, select=sel, align="average", gpus=[0, 0, 0]).run(**sl).results
    fl = np.sort(np.arange(len(traj))[slice(sl.get("start"), sl.get("stop"), sl["step"])])
    exp = O.rmsf_script(traj[np.concatenate([[0], fl])], sel, None, size=3, align="average", start=1)
    np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    assert r.n_frames == len(fl)


def test_multi_frames_xtc_atomgroup_dcd(tmp_path, traj):
    """frames= (indices / a boolean mask) with gpus= for the file and
    AtomGroup inputs, against the oracle on those frames."""
    from oracle import xtc_py
    from rmsf_amd import RMSF
    from rmsf_amd.dcd import write_dcd
    from rmsf_amd.xtc import write_xtc
    from test_gpu_multirank import _FakeAtomGroup, _FakeUniverse
    sel = np.arange(2, 700, 5)
    idx = np.array([1, 3, 5, 6, 7, 19, 30, 33, 36])
    xp = str(tmp_path / "m.xtc")
    write_xtc(xp, traj)
    q = xtc_py.read_xtc(xp)
    r = RMSF(xp, select=sel, align="average", gpus=[0, 0]).run(frames=idx).results
    exp = O.rmsf_script(q[np.concatenate([[0], idx])], sel, None, size=2, align="average", start=1)
    np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    ag = _FakeAtomGroup(_FakeUniverse(traj), sel, None)
    r = RMSF(ag, align="frame0", masses=np.ones(len(sel)), gpus=[0, 0, 0]).run(frames=idx).results
    exp = O.rmsf_script(traj[np.concatenate([[0], idx])], sel, None, size=3, align="frame0", start=1)
    np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)
    dp = str(tmp_path / "m.dcd")
    write_dcd(dp, traj)
    mask = np.zeros(len(traj), bool)
    mask[idx] = True
    for align in (None, "average"):  # streamed runs; staged into HBM for the two sweeps
        r = RMSF(dp, select=sel, align=align, gpus=[0, 0]).run(frames=mask).results
        exp = O.rmsf_script(traj[np.concatenate([[0], idx])], sel, None, size=2, align=align, start=1)
        np.testing.assert_allclose(r.rmsf, exp["rmsf"], rtol=0, atol=TOL)


@pytest.mark.parametrize("align", [None, "frame0", "average"])
def test_multi_explicit_frames(traj, align):
    """gpus= with run(frames=...): each device takes its RMSF.py:65-69 block of
    the frame list as strided runs; same result as one device."""
    from rmsf_amd import RMSF
    idx = np.array([0, 2, 4, 6, 7, 8, 13, 14, 20, 20, 29])
    idx = idx[idx < len(traj)]
    sel = np.arange(1, traj.shape[1], 3)
    one = RMSF(traj, select=sel, align=align).run(frames=idx).results
    r = RMSF(traj, select=sel, align=align, gpus=[0, 0, 0]).run(frames=idx).results
    np.testing.assert_allclose(r.rmsf, one.rmsf, rtol=0, atol=1e-9)
    assert r.n_frames == len(idx)
