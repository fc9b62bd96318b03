"""CPU tier: the frame selection of RMSF.run() -- start/stop/step or an
explicit ``frames`` list / boolean mask (MDAnalysis AnalysisBase.run) -- and
its decomposition into strided batches (``FrameList.runs``), which every
frame source reads."""
import numpy as np
import pytest

from rmsf_amd.sources import FrameList


def _expand(fl, b0, b1, max_n):
    out = []
    for first, step, n in fl.runs(b0, b1, max_n):
        assert step >= 1 and 1 <= n <= max_n
        out += [first + k * step for k in range(n)]
    return out


@pytest.mark.parametrize("sl", [(None, None, None), (3, 90, 2), (5, None, 7), (None, 40, None)])
@pytest.mark.parametrize("max_n", [1, 4, 1000])
def test_range_runs(sl, max_n):
    fl = FrameList(98, *sl)
    r = range(98)[slice(*sl)]
    assert len(fl) == len(r)
    for b0, b1 in [(0, len(r)), (1, len(r) // 2), (len(r) // 2, len(r))]:
        assert _expand(fl, b0, b1, max_n) == list(r[b0:b1])


@pytest.mark.parametrize("max_n", [1, 3, 64])
def test_explicit_runs(max_n):
    rng = np.random.default_rng(4)
    f = rng.choice(200, 80, replace=True)  # duplicates and gaps
    fl = FrameList(200, frames=f)
    want = sorted(int(x) for x in f)
    assert len(fl) == 80 and [fl[i] for i in range(80)] == want
    for b0, b1 in [(0, 80), (0, 1), (17, 63), (79, 80)]:
        assert _expand(fl, b0, b1, max_n) == want[b0:b1]


def test_explicit_arithmetic_stretches_are_single_runs():
    fl = FrameList(100, frames=[0, 2, 4, 6, 7, 8, 9, 30, 60, 90, 91])
    assert list(fl.runs(0, len(fl), 100)) == [(0, 2, 4), (7, 1, 3), (30, 30, 3), (91, 1, 1)]


def test_mask_negative_and_reversed():
    m = np.zeros(50, bool)
    m[[1, 5, 9, 13, 20]] = True
    assert _expand(FrameList(50, frames=m), 0, 5, 8) == [1, 5, 9, 13, 20]
    assert _expand(FrameList(50, frames=[-1, 0, -50]), 0, 3, 8) == [0, 0, 49]
    fl = FrameList(50, None, None, -3)  # reversed range: the same frames, ascending
    assert _expand(fl, 0, len(fl), 8) == sorted(range(50)[::-3])


def test_frame_selection_errors():
    with pytest.raises(ValueError):
        FrameList(10, 0, None, None, frames=[1, 2])
    with pytest.raises(IndexError):
        FrameList(10, frames=[3, 10])
    with pytest.raises(IndexError):
        FrameList(10, frames=[-11])
    with pytest.raises(ValueError):
        FrameList(10, frames=np.ones(9, bool))
    assert len(FrameList(10, frames=[])) == 0


def test_non_integer_frames_rejected():
    with pytest.raises(TypeError):
        FrameList(10, frames=[1.7, 2.0])
    with pytest.raises(TypeError):
        FrameList(10, frames=np.array(["1"]))
    assert len(FrameList(10, frames=[])) == 0
    assert list(FrameList(10, frames=np.array([3, 1], dtype=np.int32)).idx) == [1, 3]


def _shard(offset, rows, n_traj):
    """A DeviceSource over a CPU tensor (bounds logic only: no kernel runs)."""
    import torch

    from rmsf_amd.sources import DeviceSource

    src = DeviceSource.__new__(DeviceSource)
    src.traj = torch.zeros(rows, 4, 3)
    src.n_atoms, src.fstride, src.offset, src.n_traj = 4, 12, offset, n_traj
    src.sel_dev = None
    return src


def test_sharded_run_checks_both_ends():
    """a rank's shard holds its RMSF.py:65-69 block of the
    trajectory, but with start/step the block of the *frame list* can run
    past it -- the last frame of a run is checked, not only the first."""
    from rmsf_amd import parallel

    n_traj, world = 20, 2
    blocks = parallel.blocks(n_traj, world)
    shard = _shard(blocks[0][0], blocks[0][1] - blocks[0][0], n_traj)  # rank 0 holds frames [0, 10)
    fl = FrameList(n_traj)
    assert sum(b.n_frames for b in shard.batches(fl, *blocks[0], 100, 0)) == 10
    fl = FrameList(n_traj, start=4)                                   # 16 frames: rank 0 gets positions [0, 8)
    b0, b1 = parallel.blocks(len(fl), world)[0]                       # = frames 4..11: past the shard
    with pytest.raises(IndexError, match="frame 11"):
        list(shard.batches(fl, b0, b1, 100, 0))
    with pytest.raises(IndexError, match="frame 11"):                 # split into runs: the failing one raises
        list(shard.batches(fl, b0, b1, 4, 0))
