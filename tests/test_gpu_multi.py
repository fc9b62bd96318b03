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
    with pytest.raises(TypeError):
        RMSF(torch.tensor(traj, device="cuda"), gpus=[0, 0]).run()
    with pytest.raises(ZeroDivisionError):
        RMSF(traj, gpus=[0, 0]).run(start=5, stop=5)
    with pytest.raises(NotImplementedError):
        RMSF(traj, align="frame0", collect_rmsd=True, gpus=1).run()


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
