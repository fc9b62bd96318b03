"""GPU tier: the sharded (N>1) pipeline on one MI355X.

RCCL will not put two ranks on one device, so the two processes here share
cuda:0 over a gloo process group (gloo all-reduces/broadcasts HIP tensors).
Everything else is the product path of a real multi-GPU run: each rank holds
only its own frame shard in HBM (RMSF.py:65-69 blocks), the reference frame's
owner computes and broadcasts it, sweep 1 is all-reduced, and the exact k-way
Chan merge runs through the HIP kernels."""
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _worker(rank, size, port, align, n_frames, q):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(port, rank, size)
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        from rmsf_amd.synth import generate, motion_table
        eng = Engine(torch.device("cuda", 0))
        n_atoms = 700
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        mt = motion_table(3, n_frames)
        shard = generate(eng, n_atoms, b0, max(b1 - b0, 1), seed=2, motion=mt)[: b1 - b0]
        sel = np.arange(5, n_atoms, 3)
        src = DeviceSource(shard, sel, offset=b0, n_traj=n_frames)
        res = run_pipeline(eng, src, FrameList(n_frames), align=align)
        torch.cuda.synchronize()
        q.put((rank, res.rmsf.cpu().numpy(), res.n_local))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_frames,align", [(2, 41, "average"), (2, 41, "frame0"), (2, 30, None),
                                                 (3, 2, "average"), (3, 2, None), (3, 40, None), (3, 40, "frame0")])
def test_sharded_pipeline_two_processes(size, n_frames, align):
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table

    from conftest import spawn_ranks
    out = spawn_ranks(_worker, size, lambda r, init, q: (r, size, init, align, n_frames, q), timeout=100)
    for rank, r, n_local in out:
        assert n_local >= 0, r
    traj = SY.frames(2, 700, 0, n_frames, motion_table(3, n_frames))
    exp = O.rmsf_script(traj, np.arange(5, 700, 3), None, size=size, align=align)["rmsf"]
    assert sum(o[2] for o in out) == n_frames
    for rank, rmsf, _ in out:
        np.testing.assert_allclose(rmsf, exp, rtol=0, atol=1e-6)


class _FakeTS:
    def __init__(self, frame):
        self.frame = frame


class _FakeTrajectory:
    """Duck-typed MDAnalysis trajectory: indexing seeks and fills a shared
    float32 positions buffer (as a reader's Timestep does)."""

    def __init__(self, traj):
        self._t = traj
        self.ts = _FakeTS(0)
        self.positions = traj[0].copy()

    def __len__(self):
        return len(self._t)

    def __getitem__(self, i):
        self.ts.frame = i
        self.positions[:] = self._t[i]
        return self.ts


def _api_worker(rank, size, init, q, kind, path, align, run_kw):
    """rmsf_amd.RMSF(...).run() on one torch.distributed rank (the script-mode
    shape: every rank holds the whole input, run() takes its RMSF.py:65-69
    block; the cross-rank merge is the one-all-reduce form, its shift frame
    staged from the host or decoded from the XTC by the owner)."""
    sys.path[:0] = [ROOT, PKG]
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from oracle import synth as SY
        from rmsf_amd import RMSF
        from rmsf_amd.synth import motion_table
        sel = np.arange(3, 500, 4)
        inp = path if kind == "xtc" else SY.frames(4, 500, 0, 37, motion_table(5, 37))
        r = RMSF(inp, select=sel, align=align, batch_frames=7).run(**run_kw)
        q.put((rank, r.results.rmsf, r.results.n_frames))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["host", "xtc"])
@pytest.mark.parametrize("align,run_kw", [(None, {}), ("frame0", dict(step=2)), ("average", {}),
                                          (None, dict(frames=[1, 4, 5, 9, 10, 11, 20, 30, 36])),
                                          ("average", dict(start=30, stop=2, step=-3))])
def test_api_under_torch_distributed(tmp_path, kind, align, run_kw):
    """RMSF(host array | .xtc path).run() on 3 ranks (gloo, one GPU) against
    the oracle's mpirun -n 3 emulation of the same frame list: staged and
    XTC-decoded batches, strided / explicit / reversed frame lists, every
    alignment mode -- each through the one-all-reduce Chan merge."""
    from conftest import spawn_ranks
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from oracle import xtc_py
    from rmsf_amd.sources import FrameList
    from rmsf_amd.synth import motion_table
    from rmsf_amd.xtc import write_xtc

    traj = SY.frames(4, 500, 0, 37, motion_table(5, 37))
    path = str(tmp_path / "r.xtc")
    if kind == "xtc":
        write_xtc(path, traj)
        traj = xtc_py.read_xtc(path)
    size = 3
    out = spawn_ranks(_api_worker, size, lambda r, init, q: (r, size, init, q, kind, path, align, run_kw))
    fl = FrameList(37, **run_kw)
    frames = np.array([fl[i] for i in range(len(fl))])
    sel = np.arange(3, 500, 4)
    # trajectory frame 0 stays the reference (RMSF.py:80-87) whatever the list
    exp = O.rmsf_script(traj[np.concatenate([[0], frames])], sel, None, size=size, align=align, start=1)["rmsf"]
    for rank, rmsf, n in sorted(out, key=lambda o: o[0]):
        assert n == len(frames), rmsf
        np.testing.assert_allclose(rmsf, exp, rtol=0, atol=1e-6)


def _array_worker(rank, size, init, q, traj, align):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        eng = Engine(torch.device("cuda", 0))
        n = traj.shape[0]
        b0, b1 = parallel.blocks(n, size)[rank]
        shard = torch.tensor(traj[b0:max(b1, b0 + 1)], device=eng.device)[: b1 - b0]
        res = run_pipeline(eng, DeviceSource(shard, offset=b0, n_traj=n), FrameList(n), align=align)
        torch.cuda.synchronize()
        q.put((rank, res.rmsf.cpu().numpy(), res.mean.cpu().numpy()))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["outlier_frame0", "drift", "frozen"])
def test_shifted_merge_conditioning(case):
    """The one-all-reduce merge shifts by frame 0 (no alignment).  Because
    that shift is one of the data points, M2 >= (x_0 - mean)^2, so
    T2 <= (n+1) M2 and the subtraction T2 - T1^2/n loses at most log2(n+1)
    bits -- checked where it is hardest: frame 0 an outlier 500 A away from
    frames that move by 0.01 A, a trajectory drifting 80 A per frame, and
    frozen atoms (every frame identical: exactly 0).  3 ranks, against a
    two-pass f64 variance."""
    from conftest import spawn_ranks
    rng = np.random.default_rng(9)
    n, na = 40, 4096
    base = rng.uniform(0, 100, (na, 3))
    if case == "outlier_frame0":
        traj = base + 0.01 * rng.standard_normal((n, na, 3))
        traj[0] += 500.0
    elif case == "drift":
        traj = base + 80.0 * np.arange(n)[:, None, None] + 0.3 * rng.standard_normal((n, na, 3))
    else:
        traj = np.broadcast_to(base, (n, na, 3)).copy()
    traj = traj.astype(np.float32)
    out = spawn_ranks(_array_worker, 3, lambda r, init, q: (r, 3, init, q, traj, None))
    x = traj.astype(np.float64)
    exp = np.sqrt(((x - x.mean(0)) ** 2).sum(0).sum(1) / n)
    for rank, rmsf, mean in out:
        assert mean is not None, rmsf
        np.testing.assert_allclose(rmsf, exp, rtol=0, atol=1e-9 * max(1.0, float(exp.max())))
        np.testing.assert_allclose(mean.reshape(-1, 3), x.mean(0), rtol=0, atol=1e-9 * float(np.abs(x).max()))
        if case == "frozen":
            assert float(np.abs(rmsf).max()) == 0.0


class _FakeUniverse:
    def __init__(self, traj):
        self.trajectory = _FakeTrajectory(traj)


class _FakeAtomGroup:
    def __init__(self, u, idx, masses):
        self.universe, self._idx, self.masses = u, idx, masses

    def __len__(self):
        return len(self._idx)

    @property
    def positions(self):
        return self.universe.trajectory.positions[self._idx].copy()


def test_atomgroup_source_duck_typed():
    """The AtomGroup path (ag.universe.trajectory, ag.positions, ag.masses):
    RMSF.py's own semantics incl. mass-weighted COMs (RMSF.py:84,94)."""
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    traj = SY.frames(6, 400, 0, 23, motion_table(7, 23))
    idx = np.arange(1, 400, 5)
    masses = np.random.default_rng(0).uniform(1, 16, len(idx))
    ag = _FakeAtomGroup(_FakeUniverse(traj), idx, masses)
    r = RMSF(ag, align="average", batch_frames=5).run()
    exp = O.rmsf_script(traj, idx, masses, size=1, align="average")["rmsf"]
    np.testing.assert_allclose(r.results.rmsf, exp, rtol=0, atol=1e-6)
    assert ag.universe.trajectory.ts.frame == 22  # reference frame restored, then swept


@pytest.mark.parametrize("slots", [1, 2])
def test_stager_slot_reuse(slots):
    """Host stream through 1- and 2-slot pinned stagers (every slot reused
    many times): same answer as the device-resident path."""
    import torch
    from oracle import synth as SY
    from rmsf_amd import RMSF
    from rmsf_amd.sources import HostSource
    from rmsf_amd.pipeline import run_pipeline
    from rmsf_amd.engine import Engine
    from rmsf_amd.sources import FrameList
    traj = SY.frames(8, 300, 0, 50)
    sel = np.arange(0, 300, 2)
    eng = Engine()
    src = HostSource(traj, sel, batch_frames=3, n_slots=slots, n_threads=2)
    res = run_pipeline(eng, src, FrameList(50), align="frame0", max_batch=3)
    torch.cuda.synchronize()
    ref = RMSF(torch.tensor(traj, device="cuda"), select=sel, align="frame0").run().results.rmsf
    np.testing.assert_allclose(res.rmsf.cpu().numpy(), ref, rtol=0, atol=1e-9)


def _slab_worker(rank, size, init, q, n_atoms, n_frames):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        from rmsf_amd.synth import generate
        eng = Engine(torch.device("cuda", 0))
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        shard = generate(eng, n_atoms, b0, b1 - b0, seed=12)
        src = DeviceSource(shard, offset=b0, n_traj=n_frames)
        outs = {}
        for k in (0, 4, 3):
            res = run_pipeline(eng, src, FrameList(n_frames), merge_slabs=k)
            torch.cuda.synchronize()
            outs[k] = (res.rmsf.cpu().numpy(), res.mean.cpu().numpy(), res.m2.cpu().numpy(),
                       res.extras.get("merge_slabs", 0))
        q.put((rank, outs))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size", [2, 3])
def test_merge_slabs_bitwise(size):
    """C4's merge in atom slabs (each slab's all-reduce started while the
    next slab streams): every slab replays the whole plan's ranges and
    segments for its chunks, so the per-rank T1/T2 are the unslabbed ones bit
    for bit.  2 ranks: the summed result too (a + b = b + a); 3 ranks: the
    collective's summation order follows the message size (gloo: ~1 element
    in 10^6 moves by an ulp) -- counted here, within 1e-14 relative.  300k
    atoms: the flat plan is chunk-aligned (more chunks than workgroups), as
    at C4's 1M."""
    from conftest import spawn_ranks
    from oracle import synth as SY
    n_atoms, n_frames = 300_000, 64 * size + 1
    out = spawn_ranks(_slab_worker, size, lambda r, init, q: (r, size, init, q, n_atoms, n_frames), timeout=200)
    for rank, outs in sorted(out, key=lambda o: o[0]):
        assert isinstance(outs, dict), outs
        assert outs[0][3] == 0 and outs[4][3] == 4 and outs[3][3] == 3
        for k in (4, 3):
            for a, b in zip(outs[0][:3], outs[k][:3]):
                if size == 2:
                    np.testing.assert_array_equal(a, b)
                else:  # a few ulps where the 3-rank sum order changed
                    np.testing.assert_allclose(a, b, rtol=1e-14, atol=0)
            diff = sum(int((a != b).sum()) for a, b in zip(outs[0][:3], outs[k][:3]))
            print(f"\nsize {size} rank {rank} slabs {k}: elements differing from unslabbed: {diff} of "
                  f"{sum(a.size for a in outs[0][:3])}")
    # sampled atoms against a two-pass variance of the regenerated frames
    atoms = np.sort(np.random.default_rng(1).choice(n_atoms, 64, replace=False))
    host = SY.frames(12, n_atoms, 0, n_frames, atoms=atoms).astype(np.float64)
    exp = np.sqrt(((host - host.mean(0)) ** 2).sum(0).sum(1) / n_frames)
    np.testing.assert_allclose(out[0][1][4][0][atoms], exp, rtol=0, atol=1e-9)


def _root_worker(rank, size, init, q, n_atoms, n_frames, align, slabs):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        from rmsf_amd.synth import generate, motion_table
        eng = Engine(torch.device("cuda", 0))
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        mt = motion_table(5, n_frames) if align else None
        shard = generate(eng, n_atoms, b0, b1 - b0, seed=14, motion=mt)
        src = DeviceSource(shard, offset=b0, n_traj=n_frames)
        fl = FrameList(n_frames)
        every = run_pipeline(eng, src, fl, align=align, merge_slabs=slabs, ref_owner=0)
        root = run_pipeline(eng, src, fl, align=align, merge_slabs=slabs, ref_owner=0, merge_root=0)
        torch.cuda.synchronize()
        got = None if root.rmsf is None else [t.cpu().numpy() for t in (root.rmsf, root.mean, root.m2)]
        q.put((rank, [t.cpu().numpy() for t in (every.rmsf, every.mean, every.m2)], got,
               root.extras.get("merge_slabs", 0)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_atoms,align,slabs", [(2, 3000, None, 0), (3, 3000, "frame0", 0),
                                                      (3, 3000, "average", 0), (2, 300_000, None, 2)])
def test_merge_to_root(size, n_atoms, align, slabs):
    """RMSF.py:143's shape: the final merge as a reduce to rank 0.  Rank 0's
    result equals the all-reduce merge's (same T1/T2 summed; 2 ranks bit for
    bit, 3 ranks within the collective's summation order); the other ranks
    get None.  Also through C4's atom slabs (300k atoms)."""
    from conftest import spawn_ranks
    n_frames = 40 * size + 1
    out = spawn_ranks(_root_worker, size, lambda r, init, q: (r, size, init, q, n_atoms, n_frames, align, slabs),
                      timeout=200)
    for rank, every, got, k in sorted(out, key=lambda o: o[0]):
        assert isinstance(every, list), every
        assert k == slabs
        if rank != 0:
            assert got is None
            continue
        for a, b in zip(every, got):
            if size == 2:
                np.testing.assert_array_equal(a, b)
            else:
                np.testing.assert_allclose(a, b, rtol=1e-13, atol=1e-13)


def _scatter_worker(rank, size, init, q, n_atoms, n_frames, align):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        from rmsf_amd.synth import generate, motion_table
        eng = Engine(torch.device("cuda", 0))
        b0, b1 = parallel.blocks(n_frames, size)[rank]
        mt = motion_table(7, n_frames) if align else None
        shard = generate(eng, n_atoms, b0, b1 - b0, seed=15, motion=mt)
        src = DeviceSource(shard, offset=b0, n_traj=n_frames)
        fl = FrameList(n_frames)
        # the frame-parallel all-reduce merge (exact=False: a few-frame aligned
        # run would default to the exact path, whose merge is another form)
        every = run_pipeline(eng, src, fl, align=align, ref_owner=0, exact=False)
        sc = run_pipeline(eng, src, fl, align=align, ref_owner=0, merge_root=0, merge_scatter=True)
        torch.cuda.synchronize()
        a0, a1 = sc.extras["atom_slice"]
        # the same through the MDAnalysis-style surface
        from rmsf_amd import RMSF
        R = RMSF(src, align=align, merge_root=0, merge_scatter=True).run().results
        assert R.atom_slice == (a0, a1) and R.mean is None
        np.testing.assert_array_equal(R.slice_mean, sc.extras["slice_mean"].cpu().numpy())
        if rank == 0:
            np.testing.assert_array_equal(R.rmsf, sc.rmsf.cpu().numpy())
        else:
            assert R.rmsf is None
        q.put((rank, [t.cpu().numpy() for t in (every.rmsf, every.mean, every.m2)],
               None if sc.rmsf is None else sc.rmsf.cpu().numpy(),
               (a0, a1, sc.extras["slice_mean"].cpu().numpy(), sc.extras["slice_m2"].cpu().numpy())))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_atoms,align", [(2, 3000, None), (3, 3001, None), (2, 3000, "frame0"),
                                                (3, 2999, "average"), (4, 10, None)])
def test_merge_reduce_scatter(size, n_atoms, align):
    """The merge as a reduce-scatter by atom slices (bench --merge scatter):
    each rank finishes its slice (the last one padded when size does not
    divide the atoms) and only the RMSF is gathered to rank 0.  Rank r's
    slice of mean and M2 and rank 0's RMSF equal the all-reduce merge's: bit
    for bit with 2 ranks, within the collective's summation order with 3-4;
    against the oracle's P-rank RMSF.py within 1e-6 A."""
    from conftest import spawn_ranks
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table
    n_frames = 30 * size + 2
    out = spawn_ranks(_scatter_worker, size, lambda r, init, q: (r, size, init, q, n_atoms, n_frames, align),
                      timeout=200)
    covered = 0
    errors = [o for o in out if not isinstance(o[1], list)]
    assert not errors, errors
    for rank, every, rmsf, sl in sorted(out, key=lambda o: o[0]):
        a0, a1, mean_s, m2_s = sl
        covered += a1 - a0
        pairs = [(mean_s, every[1][a0:a1]), (m2_s, every[2][a0:a1])]
        if rank == 0:
            pairs.append((rmsf, every[0]))
        else:
            assert rmsf is None
        for got, exp in pairs:
            if size == 2:
                np.testing.assert_array_equal(got, exp)
            else:
                np.testing.assert_allclose(got, exp, rtol=1e-13, atol=1e-13)
    assert covered == n_atoms
    mt = motion_table(7, n_frames) if align else None
    traj = SY.frames(15, n_atoms, 0, n_frames, mt)
    exp = O.rmsf_script(traj, None, None, size=size, align=align)["rmsf"]
    r0 = next(o for o in out if o[0] == 0)
    np.testing.assert_allclose(r0[2], exp, rtol=0, atol=1e-6)
