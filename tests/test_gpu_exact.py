"""GPU tier: ``exact=True`` -- RMSF.py:120-146 with the reference's own
arithmetic, bit for bit.

rmsf_welford_sequential runs RMSF.py:137-138's per-frame update in frame
order with numpy's operations and roundings (the library is built without FP
contraction), rmsf_chan_merge folds the ranks with second_order_moments
(RMSF.py:36-41) in rank order, and k_finalize is RMSF.py:146.  The oracle's
rank_sweep2 / rmsf_script(align=None) are those lines restated in numpy, so
every comparison here is ``assert_array_equal`` on the float64 bit patterns
-- mean, sumsquares and RMSF -- not a tolerance.  Sizes: one and two
batches (the recurrence's k continued across them), a gathered selection,
frame subsets, host and HBM inputs, 2-3 ranks sharing the GPU over gloo."""
import numpy as np
import pytest
import torch

from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.uint64)


def _same(got, want, what):
    np.testing.assert_array_equal(_bits(got), _bits(want), err_msg=what)


@pytest.mark.parametrize("n_atoms,nf,gather", [(4096, 700, False), (1001, 333, True), (5, 40, False),
                                               (3, 1, False), (257, 4097, True),
                                               # >= 49,152 selected atoms: the atom-per-lane gather
                                               (160_000, 37, True), (150_000, 9, True)])
def test_sequential_kernel_is_rmsf_py_recurrence(n_atoms, nf, gather):
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    eng = Engine()
    traj = generate(eng, n_atoms, 0, nf, seed=5)
    host = traj.cpu().numpy()
    sel = np.sort(np.random.default_rng(2).choice(n_atoms, max(1, n_atoms // 3), replace=False)) if gather \
        else np.arange(n_atoms)
    sdev = eng.sel_tensor(sel) if gather else None
    n_sel = len(sel)
    S = O.rank_sweep2(host, sel, None, 0, nf)
    m, q = eng.empty(3 * n_sel), eng.empty(3 * n_sel)
    eng.welford_sequential(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, 0, m, q)
    # the same frames in three batches: k continues at k0
    m3, q3 = eng.empty(3 * n_sel), eng.empty(3 * n_sel)
    cuts = [0, nf // 3, (2 * nf) // 3, nf]
    for f0, f1 in zip(cuts, cuts[1:]):
        eng.welford_sequential(traj.data_ptr() + f0 * 3 * n_atoms * 4, 3 * n_atoms, f1 - f0, n_sel, sdev, f0,
                               m3, q3)
    torch.cuda.synchronize()
    for got_m, got_q, how in ((m, q, "one batch"), (m3, q3, "three batches")):
        _same(got_m.cpu().numpy(), S[1].reshape(-1), f"mean, {how}")
        _same(got_q.cpu().numpy(), S[2].reshape(-1), f"sumsquares, {how}")


@pytest.mark.parametrize("kind", ["host", "hbm"])
@pytest.mark.parametrize("run_kw,batch", [({}, None), ({}, 37), ({"start": 3, "stop": 290, "step": 4}, None),
                                          ({"frames": [0, 5, 6, 9, 100, 250]}, 2)])
def test_rmsf_exact_single_rank(kind, run_kw, batch):
    from rmsf_amd import RMSF
    n_atoms, nf = 600, 300
    traj = SY.frames(11, n_atoms, 0, nf)
    sel = np.arange(2, n_atoms, 5)
    inp = traj if kind == "host" else torch.tensor(traj, device="cuda")
    r = RMSF(inp, select=sel, exact=True, batch_frames=batch).run(**run_kw).results
    fl = O._frame_list(nf, run_kw.get("start"), run_kw.get("stop"), run_kw.get("step"))
    if "frames" in run_kw:
        fl = run_kw["frames"]
    want = O.rmsf_script(traj[fl], sel=sel, size=1, align=None)
    _same(r.mean, want["mean"], "mean")
    _same(r.sumsquares, want["m2"], "sumsquares")
    _same(r.rmsf, want["rmsf"], "rmsf")
    # the default (frame-parallel, reassociated) path agrees to rounding
    d = RMSF(inp, select=sel, batch_frames=batch).run(**run_kw).results
    np.testing.assert_allclose(d.rmsf, r.rmsf, rtol=0, atol=1e-12)


def test_rmsf_exact_rejects_splits_and_unaligned_records():
    """exact=True runs the sequential kernels (aligned runs included since
    round 6, tests/test_gpu_exact_aligned.py): no split grid, and no
    per-frame records without an alignment."""
    from rmsf_amd import RMSF
    traj = SY.frames(1, 10, 0, 5)
    with pytest.raises(ValueError):
        RMSF(traj, exact=True, n_splits=2).run()
    with pytest.raises(ValueError):
        RMSF(traj, exact=True, collect_rmsd=True).run()
    r = RMSF(traj, align="frame0", exact=True).run().results
    _same(r.rmsf, O.rmsf_script(traj, None, None, size=1, align="frame0")["rmsf"], "frame0 exact")


def _exact_worker(rank, size, init, n_frames, root, q):
    import sys

    from conftest import PKG, ROOT
    sys.path[:0] = [ROOT, PKG]
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import RMSF
        traj = SY.frames(4, 500, 0, n_frames)
        r = RMSF(traj, select=np.arange(0, 500, 2), exact=True, merge_root=root).run().results
        q.put((rank, r.rmsf, r.mean, r.sumsquares, r.block))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,n_frames,root", [(2, 61, 0), (3, 100, None), (3, 2, 1)])
def test_rmsf_exact_ranks(size, n_frames, root):
    """RMSF.py under mpirun -n size: each rank's block (RMSF.py:65-69)
    through the recurrence, the ranks folded in rank order (RMSF.py:143's
    reduce with second_order_moments), bit for bit with the oracle's
    rmsf_script(size=...); 2 frames on 3 ranks leaves rank 0 empty."""
    from conftest import spawn_ranks
    out = spawn_ranks(_exact_worker, size, lambda r, init, q: (r, size, init, n_frames, root, q), timeout=100)
    traj = SY.frames(4, 500, 0, n_frames)
    want = O.rmsf_script(traj, sel=np.arange(0, 500, 2), size=size, align=None)
    for rank, rmsf, mean, m2, block in sorted(out, key=lambda o: o[0]):
        assert not isinstance(rmsf, str), rmsf
        if root is not None and rank != root:
            assert rmsf is None and mean is None
            continue
        _same(rmsf, want["rmsf"], f"rank {rank} rmsf")
        _same(mean, want["mean"], f"rank {rank} mean")
        _same(m2, want["m2"], f"rank {rank} sumsquares")


@pytest.mark.parametrize("n_atoms,nf", [(400, 90), (240_000, 30)])  # 60,000 selected: one atom per lane
@pytest.mark.parametrize("device", [False, True])
def test_context_exact_push_is_rmsf_py_rank(device, n_atoms, nf):
    """RMSF_PUSH_EXACT through the context ABI (the torch-free boundary an
    mpi4py / C host binds): a rank's S of RMSF.py:140 bit for bit over
    several pushes (host frames through the stager in 7-frame batches, or
    HBM frames), with a gathered selection; reduced by RMSF.py's own
    second_order_moments in rank order (the oracle's chan_fold, what
    RMSF.py:143 runs on the host) they give rmsf_script(size=3)'s result.
    A checkpoint (get / set_partial) continues the recurrence exactly."""
    from rmsf_amd import parallel
    from rmsf_amd.context import PUSH_EXACT, Context
    traj = SY.frames(21, n_atoms, 0, nf)
    sel = np.arange(3, n_atoms, 4)
    x = torch.tensor(traj, device="cuda") if device else traj
    parts = []
    for b0, b1 in parallel.blocks(nf, 3):
        S = O.rank_sweep2(traj, sel, None, b0, b1)
        mid = (b0 + b1) // 2
        with Context(n_atoms, sel=sel) as c, Context(n_atoms, sel=sel) as d:
            c.set_staging(batch_frames=7, n_slots=2, n_threads=2)
            c.push(x[b0:mid], PUSH_EXACT)
            d.set_partial(*c.partial())          # checkpoint -> restore, then continue
            c.push(x[mid:b1], PUSH_EXACT)
            d.push(x[mid:b1], PUSH_EXACT)
            for ctx in (c, d):
                n, mean, m2 = ctx.partial()
                assert n == b1 - b0
                _same(mean.reshape(-1), S[1].reshape(-1), f"block {b0}-{b1} mean")
                _same(m2.reshape(-1), S[2].reshape(-1), f"block {b0}-{b1} sumsquares")
            parts.append((n, mean.reshape(-1, 3), m2.reshape(-1, 3)))
            _same(c.rmsf(), np.sqrt(S[2].sum(axis=1) / (b1 - b0)), "the context's own RMSF.py:146")
    Data = O.chan_fold(parts)
    want = O.rmsf_script(traj, sel, size=3, align=None)
    _same(np.sqrt(Data[2].sum(axis=1) / Data[0]), want["rmsf"], "rmsf, 3 ranks reduced in rank order")


def test_script_mode_exact(tmp_path):
    """rmsf_mi355x.py --align none --exact on RMSF.py's input pair (GRO +
    XTC, read natively): the script's own arithmetic on the decoded frames,
    bit for bit; --exact with alignment is refused."""
    import subprocess
    import sys

    from conftest import ROOT
    from rmsf_amd.topology import GroTopology, write_gro
    from rmsf_amd.xtc import XTCFile, write_xtc
    n_res = 40
    resids = np.repeat(np.arange(1, n_res + 1), 3)
    resnames = np.array(["ALA"] * (3 * n_res))
    names = np.tile(["N", "CA", "C"], n_res)
    x = SY.frames(31, len(names), 0, 33)
    gro, xtc, out = str(tmp_path / "s.gro"), str(tmp_path / "s.xtc"), str(tmp_path / "rmsf.npy")
    write_gro(gro, resids, resnames, names, x[0])
    write_xtc(xtc, x)
    script = f"{ROOT}/mdanalysis-mpi_amd/rmsf_mi355x.py"
    r = subprocess.run([sys.executable, script, "--topology", gro, "--trajectory", xtc, "--out", out,
                        "--align", "none", "--exact"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    sel = GroTopology(gro).select("protein and name CA")
    with XTCFile(xtc) as f:
        dec = f.read()
    _same(np.load(out), O.rmsf_script(dec, sel, None, size=1, align=None)["rmsf"], "script --exact")
    bad = subprocess.run([sys.executable, script, "--synthetic", "10", "5", "--exact"], capture_output=True,
                         text=True, timeout=120)
    assert bad.returncode != 0 and "--exact needs --align none" in bad.stderr


@pytest.mark.parametrize("inp", ["host", "shards"])
@pytest.mark.parametrize("gpus", [1, [0, 0, 0]])
def test_rmsf_exact_one_process_devices(inp, gpus):
    """RMSF(gpus=..., exact=True): each device context runs RMSF.py:137-138's
    recurrence over its RMSF.py:65-69 block (RMSF_PUSH_EXACT), the blocks
    are folded in device order by second_order_moments: rmsf_script with
    size = the device count, bit for bit.  Host input (contexts stage their
    blocks) and HBM shards (each device's frames in place, three shards of
    a 71-frame trajectory)."""
    from rmsf_amd import RMSF, parallel
    n_atoms, nf = 300, 71
    traj = SY.frames(17, n_atoms, 0, nf)
    sel = np.arange(1, n_atoms, 3)
    n_dev = 1 if gpus == 1 else len(gpus)
    if inp == "host":
        x = traj
    else:
        x = [torch.tensor(traj[b0:b1], device="cuda") for b0, b1 in parallel.blocks(nf, n_dev)]
    r = RMSF(x, select=sel, exact=True, gpus=gpus, batch_frames=9).run().results
    want = O.rmsf_script(traj, sel, None, size=n_dev, align=None)
    _same(r.rmsf, want["rmsf"], "rmsf")
    _same(r.mean, want["mean"], "mean")
    _same(r.sumsquares, want["m2"], "sumsquares")


@pytest.mark.parametrize("n_atoms,n_sel", [(64, None), (60_000, 50_000)])
def test_sequential_special_values(n_atoms, n_sel):
    """Zeros (both signs), infinities and NaNs in the frames: the fast
    division's select passes zero and infinity numerators through, NaN
    propagates -- the reference recurrence's values wherever it has a
    number, NaN wherever it has NaN.  (60,000 atoms, 50,000 selected: the
    atom-per-lane gather.)"""
    from rmsf_amd.engine import Engine
    eng = Engine()
    nf = 50
    traj = SY.frames(3, n_atoms, 0, nf)
    rng = np.random.default_rng(9)
    sel = np.arange(n_atoms) if n_sel is None else \
        np.union1d([5, 6], rng.choice(n_atoms, n_sel - 2, replace=False))[:n_sel]
    for v in (0.0, -0.0, np.inf, -np.inf, np.nan):
        k = 6 if n_sel is None else 400
        idx = rng.integers(0, nf, k), rng.integers(0, n_atoms, k), rng.integers(0, 3, k)
        traj[idx] = np.float32(v)
    traj[:, 5, 0] = 0.0            # a column that is zero throughout
    traj[:, 6, 1] = -0.0           # ... and negative zero throughout
    S = O.rank_sweep2(traj, sel, None, 0, nf)
    x = torch.tensor(traj, device="cuda")
    ns = len(sel)
    m, q = eng.empty(3 * ns), eng.empty(3 * ns)
    eng.welford_sequential(x.data_ptr(), 3 * n_atoms, nf, ns, None if n_sel is None else eng.sel_tensor(sel), 0,
                           m, q)
    torch.cuda.synchronize()
    for got, want, what in ((m.cpu().numpy(), S[1].reshape(-1), "mean"), (q.cpu().numpy(), S[2].reshape(-1),
                                                                         "sumsquares")):
        nan = np.isnan(want)
        assert np.array_equal(np.isnan(got), nan), f"{what}: NaN pattern"
        _same(got[~nan], want[~nan], what)
