"""GPU tier: host frames stored as coordinate planes (SoA, [F, 3, n_atoms] --
the north star's "synthetic in-memory SoA coordinate array", and a DCD
frame's X/Y/Z records in place) staged through rmsf_stager_stage_planes,
which interleaves the selection into the same (frame, atom, xyz) device
batches as [F, n_atoms, 3] input.  The results must be BITWISE those of the
[F, n_atoms, 3] path (itself checked against the oracle and the reference
vectors) in every mode, for selections, strides, scattered frame lists,
padded planes, the one-process multi-device path and the context ABI; and
within 1e-6 A of the C1 golden vectors (RMSF.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def c1():
    d = np.load(os.path.join(GOLDEN, "c1_synth.npz"))
    traj = SY.frames(int(d["seed"]), int(d["n_atoms"]), 0, int(d["n_frames"]), d["motion"])
    return d, traj


def _soa(traj, pad=0):
    """[F, 3, n] planes (optionally padded: plane stride n + pad floats)."""
    F, n, _ = traj.shape
    out = np.full((F, 3, n + pad), np.nan, np.float32)
    out[:, :, :n] = traj.transpose(0, 2, 1)
    return out[:, :, :n] if pad else np.ascontiguousarray(out)


def _same(a, b):
    for k in ("rmsf", "mean", "sumsquares"):
        np.testing.assert_array_equal(a.results[k], b.results[k])
    assert a.results.n_frames == b.results.n_frames


@pytest.mark.parametrize("align,tag", [(None, "none"), ("frame0", "frame0"), ("average", "average")])
@pytest.mark.parametrize("pad", [0, 5])
def test_soa_bitwise_and_golden(c1, align, tag, pad):
    from rmsf_amd import RMSF
    d, traj = c1
    soa = _soa(traj, pad)
    r_fac = RMSF(traj, select=d["sel"], align=align).run()
    r_soa = RMSF(soa, select=d["sel"], align=align, layout="soa").run()
    _same(r_fac, r_soa)
    np.testing.assert_allclose(r_soa.results.rmsf, d[f"rmsf_{tag}_P1"], rtol=0, atol=TOL)


@pytest.mark.parametrize("align", [None, "average"])
def test_soa_slices_frames_batches(c1, align):
    from rmsf_amd import RMSF
    d, traj = c1
    soa = _soa(traj)
    for kw, run in (({"batch_frames": 7}, {"start": 3, "stop": 90, "step": 2}),
                    ({}, {"frames": np.sort(np.random.default_rng(2).choice(98, 41, replace=False))}),
                    ({"batch_frames": 5}, {"frames": np.arange(0, 98, 9)})):
        a = RMSF(traj, select=d["sel"], align=align, **kw).run(**run)
        b = RMSF(soa, select=d["sel"], align=align, layout="soa", **kw).run(**run)
        _same(a, b)


def test_soa_all_atoms_large():
    """Every atom of a 60k-atom frame set (the contiguous gather, several
    65,536-atom pieces per frame in the stager's pool at 150k)."""
    from rmsf_amd import RMSF
    for n in (60_000, 150_000):
        traj = SY.frames(9, n, 0, 12, None)
        _same(RMSF(traj).run(), RMSF(_soa(traj), layout="soa").run())


@pytest.mark.parametrize("align", [None, "frame0", "average"])
def test_soa_multi_device_path(c1, align):
    """gpus=1: the context ABI's rmsf_push_frame_planes."""
    from rmsf_amd import RMSF
    d, traj = c1
    a = RMSF(traj, select=d["sel"], align=align, gpus=1).run()
    b = RMSF(_soa(traj), select=d["sel"], align=align, layout="soa", gpus=1).run()
    _same(a, b)
    a = RMSF(traj, select=d["sel"], align=align, gpus=1).run(frames=[1, 5, 6, 40, 41, 42, 97])
    b = RMSF(_soa(traj), select=d["sel"], align=align, layout="soa", gpus=1).run(frames=[1, 5, 6, 40, 41, 42, 97])
    _same(a, b)


def test_soa_context_push(c1):
    """push_planes of contiguous planes, of a transposed VIEW of the rows
    (strides the stager cannot walk: copied first) and of padded
    planes (a wider plane stride, walked in place) all equal push_rows."""
    from rmsf_amd.context import PUSH_WELFORD, Context
    d, traj = c1
    soa = _soa(traj)
    wide = np.zeros((traj.shape[0], 3, traj.shape[1] + 5), dtype=np.float32)
    wide[:, :, :traj.shape[1]] = soa
    views = [("rows", traj), ("planes", soa), ("transposed view", traj.transpose(0, 2, 1)),
             ("padded planes", wide[:, :, :traj.shape[1]])]
    out = []
    for name, arr in views:
        c = Context(traj.shape[1], d["sel"])
        rows = np.array([0, 3, 4, 5, 50, 97])
        if name == "rows":
            c.push_rows(arr, rows, PUSH_WELFORD)
        else:
            c.push_planes(arr, rows, PUSH_WELFORD)
        out.append(c.partial())
        c.close()
    for o in out[1:]:
        assert o[0] == 6
        np.testing.assert_array_equal(out[0][1], o[1])
        np.testing.assert_array_equal(out[0][2], o[2])


@pytest.mark.parametrize("box", [None, (60.0, 90.0, 60.0, 90.0, 90.0, 60.0)])
@pytest.mark.parametrize("align", [None, "average"])
def test_dcd_planes_path_bitwise(tmp_path, c1, box, align, monkeypatch):
    """A native DCD staged from its mapped X/Y/Z records equals the read()
    path (the same file with the plane path switched off) and the array."""
    from rmsf_amd import RMSF
    from rmsf_amd.dcd import DCDFile, write_dcd
    d, traj = c1
    p = str(tmp_path / "c1.dcd")
    write_dcd(p, traj, box=box)
    fl = np.sort(np.random.default_rng(4).choice(98, 30, replace=False))
    got = [RMSF(p, select=d["sel"], align=align).run(), RMSF(p, select=d["sel"], align=align).run(frames=fl)]
    monkeypatch.setattr(DCDFile, "plane_ptrs", lambda self, frames: None)
    want = [RMSF(p, select=d["sel"], align=align).run(), RMSF(p, select=d["sel"], align=align).run(frames=fl)]
    for a, b in zip(got, want):
        _same(a, b)
    _same(got[0], RMSF(traj, select=d["sel"], align=align).run())


def test_soa_bad_inputs(c1):
    import torch

    from rmsf_amd import RMSF
    d, traj = c1
    with pytest.raises(ValueError, match="SoA trajectory"):
        RMSF(traj, layout="soa").run()  # [F, n, 3] is not planes
    with pytest.raises(ValueError, match="SoA trajectory"):
        RMSF(torch.zeros(2, 5, 3, device="cuda"), layout="soa").run()
    with pytest.raises(ValueError, match="non-overlapping"):
        RMSF(torch.zeros(30, device="cuda").as_strided((2, 3, 5), (15, 2, 1)), layout="soa").run()
    with pytest.raises(ValueError, match="layout"):
        RMSF(traj, layout="aos")


@pytest.mark.parametrize("align", [None, "frame0", "average"])
@pytest.mark.parametrize("pad", [0, 7])
def test_device_soa_bitwise(c1, align, pad):
    """HBM-resident planes [F, 3, n] (rmsf_gather_planes into compact
    batches) against the host row array streamed in batches of the same
    frames (the stager's compact batches): the same device batches, so the
    same bits -- for ranges, steps and a scattered frame list."""
    import torch

    from rmsf_amd import RMSF
    d, traj = c1
    dev = torch.tensor(_soa(traj, pad) if not pad else np.ascontiguousarray(
        np.pad(traj.transpose(0, 2, 1), ((0, 0), (0, 0), (0, pad)))), device="cuda")
    if pad:
        dev = dev[:, :, :traj.shape[1]]
    rows_dev = torch.tensor(traj, device="cuda")
    for bf, run in ((11, {}), (7, {"start": 3, "stop": 90, "step": 2}),
                    (13, {"frames": np.sort(np.random.default_rng(5).choice(98, 40, replace=False))})):
        b = RMSF(dev, select=d["sel"], align=align, layout="soa", batch_frames=bf).run(**run)
        if align is None and "frames" not in run:
            # unaligned with a selection: planes read in place by the one-atom-per-lane kernel, as
            # HBM rows with the same selection are
            a = RMSF(rows_dev, select=d["sel"], align=align, batch_frames=bf).run(**run)
        else:
            a = RMSF(traj, select=d["sel"], align=align, batch_frames=bf).run(**run)
        _same(a, b)
    r = RMSF(dev, select=d["sel"], align=align, layout="soa").run()
    tag = {None: "none", "frame0": "frame0", "average": "average"}[align]
    np.testing.assert_allclose(r.results.rmsf, d[f"rmsf_{tag}_P1"], rtol=0, atol=TOL)


def test_device_soa_all_atoms():
    """Every atom (no selection), 50,001 atoms (3 n not a multiple of 4, so
    not read in place): the planes gather's identity path, bitwise."""
    import torch

    from rmsf_amd import RMSF
    traj = SY.frames(21, 50_001, 0, 30, None)
    dev = torch.tensor(_soa(traj), device="cuda")
    _same(RMSF(traj, batch_frames=9).run(), RMSF(dev, layout="soa", batch_frames=9).run())


@pytest.mark.parametrize("n_atoms", [4000, 3001])
def test_device_planes_in_place(n_atoms):
    """Unaligned runs over contiguous planes with no selection read the planes
    in place (per-coordinate statistics in plane order, permuted to (atom,
    xyz) at the end): the rows path's results within f64 rounding (the
    coordinates sit in different chunks, so the folds round differently),
    for the whole list, a step and a scattered list.  n_atoms = 3001 makes
    3 n odd of 4: the gather path, bitwise."""
    import torch

    from rmsf_amd import RMSF
    from rmsf_amd.sources import DeviceSource
    traj = SY.frames(17, n_atoms, 0, 70, None)
    dev = torch.tensor(_soa(traj), device="cuda")
    assert DeviceSource(dev, layout="soa").native_planes == (n_atoms % 4 == 0)
    for run in ({}, {"start": 1, "stop": 69, "step": 3},
                {"frames": np.sort(np.random.default_rng(8).choice(70, 25, replace=False))}):
        a = RMSF(traj).run(**run)
        b = RMSF(dev, layout="soa").run(**run)
        for k in ("rmsf", "mean", "sumsquares"):
            np.testing.assert_allclose(a.results[k], b.results[k], rtol=1e-13, atol=1e-13)


def _planes_rank_worker(rank, size, init, q, n_atoms, n_frames, root, pad=0, slabs=None):
    import sys

    from conftest import PKG, ROOT
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
        planes = generate(eng, n_atoms + pad, b0, b1 - b0, seed=19).transpose(1, 2).contiguous()
        if pad:  # padded planes: a view of the first n_atoms of each wider plane (plane stride > n_atoms)
            planes = planes[:, :, :n_atoms]
        src = DeviceSource(planes, offset=b0, n_traj=n_frames, layout="soa")
        assert src.native_planes == (pad == 0)
        res = run_pipeline(eng, src, FrameList(n_frames), merge_root=root, merge_slabs=slabs)
        torch.cuda.synchronize()
        q.put((rank, None if res.rmsf is None else res.rmsf.cpu().numpy(), res.extras.get("merge_slabs", 0)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_atoms,root,pad,slabs", [(2, 4000, None, 0, None), (3, 4000, 0, 0, None),
                                                         (2, 1_000_000, None, 0, None), (2, 1_000_000, None, 36, None),
                                                         (2, 300_000, 0, 4, 2), (3, 4000, None, 8, 2)])
def test_device_planes_in_place_ranks(size, n_atoms, root, pad, slabs):
    """The same over gloo ranks sharing the GPU: the merge's shift (frame 0 of
    the list, broadcast) stays in plane order with the statistics; 1M atoms:
    the merge in atom slabs.  Padded planes (a plane stride wider than the
    atom count) are read through the plane kernels and never take
    the flat slab path, which reads each frame as 3n contiguous floats; their
    merge runs unslabbed.  Against a two-pass variance of the regenerated
    frames on sampled atoms (the generator's atoms 0..n-1 of the wider
    trajectory are the same values)."""
    from conftest import spawn_ranks
    n_frames = 20 * size + 3
    out = spawn_ranks(_planes_rank_worker, size,
                      lambda r, init, q: (r, size, init, q, n_atoms, n_frames, root, pad, slabs), timeout=200)
    atoms = np.sort(np.random.default_rng(2).choice(n_atoms, 64, replace=False))
    host = SY.frames(19, n_atoms, 0, n_frames, atoms=atoms).astype(np.float64)
    exp = np.sqrt(((host - host.mean(0)) ** 2).sum(0).sum(1) / n_frames)
    for rank, rmsf, k in out:
        assert k != -1, rmsf
        if root is not None and rank != root:
            assert rmsf is None
            continue
        np.testing.assert_allclose(rmsf[atoms], exp, rtol=0, atol=1e-9)
        if pad:
            assert k == 0
        elif n_atoms >= 1_000_000:
            assert k == 2


@pytest.mark.parametrize("align", ["frame0", "average"])
@pytest.mark.parametrize("n_atoms,masses", [(4000, False), (4000, True), (3001, False)])
def test_device_planes_aligned_in_place(align, n_atoms, masses):
    """Aligned sweeps read HBM planes in place (rmsf_superpose_planes: the
    float4 plane staging for 4-aligned planes, the element path otherwise;
    rmsf_accumulate_balanced_planes): the same tiles, sums and transforms as
    the row layout, so the same bits as the host rows streamed in batches of
    the same frames."""
    import torch

    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    traj = SY.frames(23, n_atoms, 0, 60, motion_table(6, 60))
    m = np.random.default_rng(3).uniform(1, 16, n_atoms) if masses else None
    dev = torch.tensor(_soa(traj), device="cuda")
    for bf, run in ((60, {}), (9, {"start": 2, "stop": 59, "step": 3})):
        a = RMSF(traj, align=align, masses=m, batch_frames=bf, collect_rmsd=True).run(**run)
        b = RMSF(dev, align=align, masses=m, layout="soa", batch_frames=bf, collect_rmsd=True).run(**run)
        _same(a, b)
        np.testing.assert_array_equal(a.results.rmsd, b.results.rmsd)
