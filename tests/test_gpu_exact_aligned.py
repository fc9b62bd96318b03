"""GPU tier: ``exact=True`` on the ALIGNED path -- RMSF.py:80-146 with the
reference's own summation orders, bit for bit.

rmsf_reference_setup_sequential (RMSF.py:84-85 / 111 + 117-118),
rmsf_superpose_sequential (RMSF.py:94-97 / 127-131 + get_rotation_matrix,
one lane per frame: the COM and qcprot's InnerProduct atom by atom) and
rmsf_accumulate_sequential (RMSF.py:99-103 / 133-138, one lane per atom,
frames in order) reproduce each statement's own rounding, so every
comparison here is ``assert_array_equal`` on float64 bit patterns against
  * tests/golden/reference_literal.npz -- RMSF.py's own statements executed
    at its literal input shape (47,681 atoms, 214 CA, 10 frames; also 2 and
    4 frames), P = 1 and 2 (two gloo ranks sharing the GPU);
  * the oracle's restatement (rmsf_script) on other shapes, selections,
    masses, frame subsets, batch splits and sources.
The default (frame-parallel) aligned path is checked at the literal shape
against the north star's 1e-6 A, and its margin printed."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, PKG, ROOT
from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64)).view(np.uint64)


def _same(got, want, what):
    np.testing.assert_array_equal(_bits(got), _bits(want), err_msg=what)


@pytest.fixture(scope="module")
def lit():
    return np.load(os.path.join(GOLDEN, "reference_literal.npz"))


@pytest.fixture(scope="module")
def lit_traj(lit):
    return SY.frames(int(lit["seed"]), int(lit["n_atoms"]), 0, int(lit["frames"].max()), lit["motion"])


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("nf", [2, 4, 10])
def test_literal_shape_exact_bit_for_bit(lit, lit_traj, nf, where):
    """RMSF.py's input shape, one rank: exact=True equals the reference's
    statements bit for bit -- RMSF, mean, sumsquares and the average."""
    from rmsf_amd import RMSF
    t = lit_traj[:nf]
    x = torch.tensor(t, device="cuda") if where == "device" else t
    r = RMSF(x, select=lit["sel"], masses=lit["masses"], align="average", exact=True).run().results
    for k, got in (("rmsf", r.rmsf), ("mean", r.mean), ("m2", r.sumsquares), ("average", r.average)):
        _same(got, lit[f"{k}_F{nf}_P1"], f"{k}, {nf} frames")


@pytest.mark.parametrize("nf", [2, 4, 10])
def test_literal_shape_default_is_exact(lit, lit_traj, nf, monkeypatch):
    """The product default (exact=None) at RMSF.py's shape: an aligned run of
    fewer than AUTO_EXACT_FRAMES frames takes the exact path -- the
    reference statements' bits.  The frame-parallel path (exact=False) is
    within one f32 rounding flip of an aligned coordinate: printed, and
    bounded by ulp(x)/sqrt(N) (<= 1.53e-5 A / sqrt(N) below 256 A)."""
    from rmsf_amd import RMSF
    monkeypatch.delenv("RMSF_AUTO_EXACT_FRAMES", raising=False)  # the product default
    t = torch.tensor(lit_traj[:nf], device="cuda")
    r = RMSF(t, select=lit["sel"], masses=lit["masses"], align="average").run().results
    for k, got in (("rmsf", r.rmsf), ("mean", r.mean), ("m2", r.sumsquares), ("average", r.average)):
        _same(got, lit[f"{k}_F{nf}_P1"], f"default, {k}, {nf} frames")
    f = RMSF(t, select=lit["sel"], masses=lit["masses"], align="average", exact=False).run().results
    d = np.abs(f.rmsf - lit[f"rmsf_F{nf}_P1"]).max()
    da = np.abs(f.average - lit[f"average_F{nf}_P1"]).max()
    print(f"\nliteral shape, {nf} frames: frame-parallel max |dRMSF| {d:.3e} A, max |daverage| {da:.3e} A")
    assert d <= 3 * 1.53e-5 / np.sqrt(nf) and da <= 1.53e-5


def _lit_worker(rank, size, init, q, nf):
    sys.path[:0] = [ROOT, PKG]
    import torch
    import torch.distributed as dist

    from conftest import init_gloo
    init_gloo(init, rank, size)
    try:
        from rmsf_amd import RMSF, parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.sources import DeviceSource
        from rmsf_amd.synth import generate
        lit = np.load(os.path.join(GOLDEN, "reference_literal.npz"))
        eng = Engine(torch.device("cuda", 0))
        b0, b1 = parallel.blocks(nf, size)[rank]
        shard = generate(eng, int(lit["n_atoms"]), b0, max(b1 - b0, 1), seed=int(lit["seed"]),
                         motion=lit["motion"])[: b1 - b0]
        src = DeviceSource(shard, lit["sel"], offset=b0, n_traj=nf)
        r = RMSF(src, masses=lit["masses"], align="average", exact=True).run().results
        q.put((rank, r.rmsf, r.mean, r.sumsquares, r.average))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nf", [2, 10])
def test_literal_shape_exact_two_ranks(lit, nf):
    """``mpirun -n 2`` at RMSF.py's shape: two ranks (gloo, sharing the GPU),
    each holding only its RMSF.py:65-69 block; frame 0's owner computes the
    first reference, sweep 1's sums meet in rank order (RMSF.py:110 -- any
    order for two ranks), the partials in comm.reduce's order: every rank's
    result equals the reference statements' P = 2 run bit for bit."""
    from conftest import spawn_ranks
    out = spawn_ranks(_lit_worker, 2, lambda r, init, q: (r, 2, init, q, nf), timeout=150)
    for rank, rmsf, mean, m2, avg in out:
        assert mean is not None, rmsf
        _same(rmsf, lit[f"rmsf_F{nf}_P2"], f"rank {rank} rmsf")
        _same(mean, lit[f"mean_F{nf}_P2"], f"rank {rank} mean")
        _same(m2, lit[f"m2_F{nf}_P2"], f"rank {rank} sumsquares")
        _same(avg, lit[f"average_F{nf}_P2"], f"rank {rank} average")


# shape, selection, masses, frame subset, batch
CASES = [
    dict(n_atoms=600, nf=40, sel="every4", masses=None, align="average", batch=None, run={}),
    dict(n_atoms=600, nf=40, sel="every4", masses="het", align="frame0", batch=7, run={}),
    dict(n_atoms=3341, nf=98, sel="random214", masses="ca", align="average", batch=30, run={}),
    dict(n_atoms=3341, nf=98, sel="random214", masses=None, align="frame0", batch=None,
         run={"start": 3, "stop": 90, "step": 2}),
    dict(n_atoms=2000, nf=5, sel="all", masses=None, align="average", batch=2, run={}),
    dict(n_atoms=20000, nf=12, sel="all", masses="het", align="average", batch=None, run={}),
    dict(n_atoms=50000, nf=3, sel="every3", masses=None, align="frame0", batch=None, run={}),
    dict(n_atoms=700, nf=33, sel="all", masses=None, align="average", batch=None, run={"frames": [0, 4, 5, 17, 30]}),
    dict(n_atoms=300, nf=1, sel="all", masses=None, align="average", batch=None, run={}),
]


def _case(c):
    from rmsf_amd.synth import motion_table
    n = c["n_atoms"]
    traj = SY.frames(7, n, 0, c["nf"], motion_table(8, c["nf"]))
    sel = {"all": np.arange(n), "every4": np.arange(1, n, 4), "every3": np.arange(0, n, 3),
           "random214": np.sort(np.random.default_rng(9).choice(n, 214, replace=False))}[c["sel"]]
    masses = {None: None, "ca": np.full(len(sel), 12.011),
              "het": np.random.default_rng(10).uniform(1.0, 16.0, len(sel))}[c["masses"]]
    return traj, sel, masses


@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_exact_aligned_vs_oracle(ci, where):
    from rmsf_amd import RMSF
    c = CASES[ci]
    traj, sel, masses = _case(c)
    x = torch.tensor(traj, device="cuda") if where == "device" else traj
    r = RMSF(x, select=sel, masses=masses, align=c["align"], exact=True, batch_frames=c["batch"],
             collect_rmsd=True).run(**c["run"]).results
    run = c["run"]
    if "frames" in run:
        # ref_frame is a TRAJECTORY frame (RMSF.py:63,83): prepend it so the
        # oracle's traj[0] is that frame, then run over the listed frames
        sub = traj[run["frames"]]
        want = O.rmsf_script(np.concatenate([traj[:1], sub]), sel, masses, size=1, align=c["align"], start=1)
    else:
        want = O.rmsf_script(traj, sel, masses, size=1, align=c["align"], start=run.get("start"),
                             stop=run.get("stop"), step=run.get("step"))
    _same(r.rmsf, want["rmsf"], "rmsf")
    _same(r.mean, want["mean"], "mean")
    _same(r.sumsquares, want["m2"], "sumsquares")
    if c["align"] == "average":
        _same(r.average, want["average"], "average")


@pytest.mark.parametrize("gathered", [False, True])
@pytest.mark.parametrize("n_sel", [1, 2, 3, 63, 64, 65, 255, 256, 257, 511, 512, 513, 769])
def test_exact_aligned_block_edges(n_sel, gathered):
    """The serial sums run 256 atoms per block in one wave (wave_seq_sum:
    whole blocks, a two-block loop, a partial last block); selections on
    either side of every block edge equal the oracle bit for bit."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    nf = 6
    n_atoms = 3 * n_sel + 1 if gathered else n_sel
    traj = SY.frames(61, n_atoms, 0, nf, motion_table(62, nf))
    sel = np.arange(1, n_atoms, 3)[:n_sel] if gathered else np.arange(n_sel)
    m = np.random.default_rng(63).uniform(1.0, 16.0, n_sel)
    for align in ("frame0", "average"):
        r = RMSF(torch.tensor(traj, device="cuda"), select=sel, masses=m, align=align, exact=True).run().results
        want = O.rmsf_script(traj, sel, m, size=1, align=align)
        _same(r.rmsf, want["rmsf"], f"rmsf {align}")
        _same(r.mean, want["mean"], f"mean {align}")
        if align == "average":
            _same(r.average, want["average"], "average")


@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("align", ["frame0", "average"])
def test_exact_aligned_graph_and_split_superpose(align, overlap, monkeypatch):
    """The exact aligned run recorded as a hipGraph (CapturedPipeline: its
    reference chains on a side stream beside the frames' COM chains) replays
    the eager run bit for bit, and the split superposition
    (rmsf_frame_com_sequential + rmsf_superpose_sequential_from_com) writes
    the records of rmsf_superpose_sequential bit for bit."""
    from rmsf_amd._lib import RMSF_XFORM_DOUBLES
    from rmsf_amd.engine import Engine
    from rmsf_amd import pipeline as PL
    from rmsf_amd.pipeline import CapturedPipeline, run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList
    from rmsf_amd.synth import motion_table
    if overlap:  # the reference's chains on the side stream at this small size too
        monkeypatch.setattr(PL, "EXACT_OVERLAP_MIN_ATOMS", 0)
    n, nf = 3000, 37
    traj = torch.tensor(SY.frames(71, n, 0, nf, motion_table(72, nf)), device="cuda")
    sel = np.arange(2, n, 5)
    m = np.random.default_rng(73).uniform(1.0, 16.0, len(sel))
    eng = Engine()
    src, fl = DeviceSource(traj, sel), FrameList(nf)
    eager = run_pipeline(eng, src, fl, align=align, masses=m, exact=True)
    cap = CapturedPipeline(eng, src, fl, align=align, masses=m, exact=True)
    for _ in range(2):
        r = cap.replay()
        torch.cuda.synchronize()
        _same(r.rmsf.cpu().numpy(), eager.rmsf.cpu().numpy(), "graph replay")
    want = O.rmsf_script(traj.cpu().numpy(), sel, m, size=1, align=align)
    _same(eager.rmsf.cpu().numpy(), want["rmsf"], "eager vs oracle")
    ns = len(sel)
    st = eng.sel_tensor(sel)
    md = torch.tensor(m, device="cuda")
    mt = float(np.asarray(m, dtype=np.float64).sum())
    ref, info = eng.reference_setup(ns, frame_ptr=traj.data_ptr(), sel=st, masses=md)
    a = eng.empty(nf, RMSF_XFORM_DOUBLES)
    b = eng.empty(nf, RMSF_XFORM_DOUBLES)
    eng.superpose_seq(traj.data_ptr(), 3 * n, nf, ns, st, md, mt, ref, info, a)
    eng.frame_com_seq(traj.data_ptr(), 3 * n, nf, ns, st, md, mt, b)
    eng.superpose_seq_from_com(traj.data_ptr(), 3 * n, nf, ns, st, ref, info, b)
    torch.cuda.synchronize()
    _same(b.cpu().numpy(), a.cpu().numpy(), "split superposition")


@pytest.mark.parametrize("n_atoms,step,masses", [(3000, 5, True), (20000, 1, False), (60000, 3, True)])
def test_exact_split_entry_points(n_atoms, step, masses):
    """The halves the side stream runs, against the whole calls, bit for bit:
    rmsf_reference_centre_sequential + rmsf_reference_sums_sequential ==
    rmsf_reference_setup_sequential (from a frame and from sweep-1 sums),
    and rmsf_inner_product_sequential + rmsf_superpose_sequential_qcp ==
    rmsf_superpose_sequential_from_com -- below and above the 16,384 atoms
    from which the reference's fill and centring run grid-wide."""
    from rmsf_amd._lib import RMSF_XFORM_DOUBLES
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import motion_table
    nf = 6
    traj = torch.tensor(SY.frames(81, n_atoms, 0, nf, motion_table(82, nf)), device="cuda")
    sel = np.arange(1, n_atoms, step) if step > 1 else None
    ns = n_atoms if sel is None else len(sel)
    m = np.random.default_rng(83).uniform(1.0, 16.0, ns) if masses else None
    md = torch.tensor(m, device="cuda") if masses else None
    mt = float(m.sum()) if masses else float(ns)
    eng = Engine()
    st = eng.sel_tensor(sel) if sel is not None else None
    marks = []  # (the record is info[:16]; the rest is the frame-parallel setup's scratch)
    _, r1, i1 = eng.reference_setup_seq(ns, mt, frame_ptr=traj.data_ptr(), sel=st, masses=md)
    _, r2, i2 = eng.reference_setup_seq(ns, mt, frame_ptr=traj.data_ptr(), sel=st, masses=md,
                                        after_centre=lambda: marks.append(1))
    total = (traj[:, torch.as_tensor(sel, device="cuda")] if sel is not None else traj).to(torch.float64).sum(0).reshape(-1).contiguous()
    a1, r3, i3 = eng.reference_setup_seq(ns, mt, total=total, n_frames=float(nf), masses=md)
    a2, r4, i4 = eng.reference_setup_seq(ns, mt, total=total, n_frames=float(nf), masses=md,
                                         after_centre=lambda: marks.append(2))
    x1 = eng.empty(nf, RMSF_XFORM_DOUBLES)
    x2 = eng.empty(nf, RMSF_XFORM_DOUBLES)
    fs = 3 * n_atoms
    eng.frame_com_seq(traj.data_ptr(), fs, nf, ns, st, md, mt, x1)
    x2.copy_(x1)
    eng.superpose_seq_from_com(traj.data_ptr(), fs, nf, ns, st, r1, i1, x1)
    eng.inner_product_seq(traj.data_ptr(), fs, nf, ns, st, r1, x2)
    eng.superpose_seq_qcp(nf, ns, i1, x2)
    torch.cuda.synchronize()
    assert marks == [1, 2]
    for got, want, what in ((r2, r1, "ref"), (i2[:16], i1[:16], "record"), (r4, r3, "ref, average"),
                            (i4[:16], i3[:16], "record, average"), (a2, a1, "average"), (x2, x1, "records")):
        _same(got.cpu().numpy(), want.cpu().numpy(), what)
    # and the oracle's reference (RMSF.py:84-85): COM atom by atom, centred
    xs = traj[0].cpu().numpy()[sel] if sel is not None else traj[0].cpu().numpy()
    com, rc = O.centred_reference(xs, m)
    _same(i1.cpu().numpy()[:3], np.asarray(com), "ref_com vs oracle")
    _same(r1.cpu().numpy(), rc, "centred ref vs oracle")


@pytest.mark.parametrize("align", ["frame0", "average"])
def test_exact_transforms_and_rmsd(align):
    """The per-frame records of the last sweep: rotation, mobile COM and the
    QCP rmsd equal the oracle's CalcRMSDRotationalMatrix on the same frame
    against the same reference, bit for bit."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    n, nf = 900, 17
    traj = SY.frames(3, n, 0, nf, motion_table(4, nf))
    sel = np.arange(0, n, 2)
    m = np.random.default_rng(5).uniform(1.0, 16.0, len(sel))
    r = RMSF(torch.tensor(traj, device="cuda"), select=sel, masses=m, align=align, exact=True,
             collect_transforms=True, collect_rmsd=True).run().results
    if align == "frame0":
        ref_com, ref_c = O.centred_reference(traj[0][sel], m)
    else:
        avg = O.rmsf_script(traj, sel, m, size=1, align="average")["average"]
        ref_com, ref_c = O.centred_reference(avg, m)
    for f in range(nf):
        p = traj[f][sel]
        com = O.center_of_mass(p, m)
        rot = np.zeros(9)
        rmsd = O.CalcRMSDRotationalMatrix(ref_c, p.astype(np.float64) - com, len(sel), rot, None)
        _same(r.transforms[f, :9], rot, f"rotation, frame {f}")
        _same(r.transforms[f, 9:12], com, f"COM, frame {f}")
        _same(r.transforms[f, 12], rmsd, f"rmsd, frame {f}")
        _same(r.rmsd[f], rmsd, f"results.rmsd, frame {f}")


def test_sequential_sum_batches_and_gather():
    """rmsf_accumulate_sequential (SUM, aligned) continues k across batches
    and reads a gathered selection: the sweep-1 sums equal RMSF.py:103's
    frame-order sum (oracle rank_sweep1) bit for bit."""
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_XFORM_DOUBLES
    eng = Engine()
    n, nf = 5000, 23
    mt = motion_table(6, nf)
    dev = generate(eng, n, 0, nf, seed=12, motion=mt)
    traj = dev.cpu().numpy()
    sel = np.sort(np.random.default_rng(1).choice(n, 777, replace=False))
    sd = eng.sel_tensor(sel)
    mtot = float(len(sel))
    _, ref, info = eng.reference_setup_seq(len(sel), mtot, frame_ptr=dev.data_ptr(), sel=sd)
    xf = eng.empty(nf, RMSF_XFORM_DOUBLES)
    eng.superpose_seq(dev.data_ptr(), 3 * n, nf, len(sel), sd, None, mtot, ref, info, xf)
    s = eng.zeros(3 * len(sel))
    for f0, f1 in ((0, 5), (5, 6), (6, nf)):
        eng.accumulate_seq(dev.data_ptr() + 4 * 3 * n * f0, 3 * n, f1 - f0, len(sel), sd, xf[f0:f1], info,
                           RMSF_MODE_SUM, f0, s, None)
    torch.cuda.synchronize()
    ref_com, ref_c = O.centred_reference(traj[0][sel])
    _same(ref.cpu().numpy().reshape(-1), ref_c.reshape(-1), "reference")
    want = O.rank_sweep1(traj, sel, None, 0, nf, ref_c, ref_com)
    _same(s.cpu().numpy(), want.reshape(-1), "sweep-1 sums")


def test_default_and_exact_agree():
    """The frame-parallel aligned path and the exact one agree far inside
    the tolerance on a many-frame run (where a flip weighs ulp/N)."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    n, nf = 4000, 300
    traj = torch.tensor(SY.frames(21, n, 0, nf, motion_table(22, nf)), device="cuda")
    sel = np.arange(0, n, 7)
    a = RMSF(traj, select=sel, align="average").run().results
    b = RMSF(traj, select=sel, align="average", exact=True).run().results
    assert np.abs(a.rmsf - b.rmsf).max() < 1e-9


@pytest.mark.parametrize("shape", [(3000, 50, 3, 10), (6000, 150, 1, 13)])
@pytest.mark.parametrize("resident", [True, False])
@pytest.mark.parametrize("align", ["frame0", "average"])
def test_compacted_sparse_selection_same_bits(align, resident, shape, monkeypatch):
    """Round 6 (verdict item 2): over a sparse gathered selection the aligned
    path writes the selected rows out once (rmsf_superpose_compact) and the
    later passes read them dense.  A gather is an exact copy and the dense
    kernels run the same arithmetic, so the results are bit-identical to the
    re-gathering path -- whole block resident (RMSF.py's second sweep reads
    it with no gather) or per batch."""
    from rmsf_amd import RMSF
    from rmsf_amd import pipeline as PL
    from rmsf_amd.synth import motion_table
    n, nf, first, stride = shape  # 300 atoms (rows of 900 floats), 462 (1,386 -> padded to 1,388)
    sel = np.arange(first, n, stride)
    if not resident:
        monkeypatch.setattr(PL._Compactor, "max_bytes", (3 * len(sel) + 3) // 4 * 4 * 4 * 30)  # 30 padded rows
    traj = torch.tensor(SY.frames(41, n, 0, nf, motion_table(42, nf)), device="cuda")
    m = np.random.default_rng(43).uniform(1.0, 16.0, len(sel))
    from rmsf_amd.engine import Engine
    from rmsf_amd.sources import DeviceSource, FrameList
    eng = Engine()
    out = {}
    for compact in (False, True):
        res = PL.run_pipeline(eng, DeviceSource(traj, sel), FrameList(nf), align=align, masses=m, compact=compact,
                              collect_rmsd=True, max_batch=23)
        torch.cuda.synchronize()
        out[compact] = {k: getattr(res, k).cpu().numpy() for k in ("rmsf", "mean", "m2", "rmsd")}
        if align == "average":
            out[compact]["average"] = res.average.cpu().numpy()
    # and the RMSF class picks compaction by itself at this density (1 in 10)
    r = RMSF(traj, select=sel, masses=m, align=align, batch_frames=23).run().results
    _same(r.rmsf, out[True]["rmsf"], "RMSF class")
    for k, v in out[False].items():
        _same(out[True][k], v, k)
    want = O.rmsf_script(traj.cpu().numpy(), sel, m, size=1, align=align)
    np.testing.assert_allclose(out[True]["rmsf"], want["rmsf"], rtol=0, atol=TOL)


@pytest.mark.parametrize("masses", [False, True])
@pytest.mark.parametrize("pitch", ["packed", "padded", "odd"])
@pytest.mark.parametrize("shape", [(2000, 64, 0, 10), (5000, 131, 2, 11), (700, 7, 5, 3)])
def test_superpose_compact_kernel(shape, pitch, masses):
    """rmsf_superpose_compact at the kernel level: the transform records are
    bit-identical to rmsf_superpose's over the same gathered rows, every
    copied row equals the selected coordinates, and nothing outside the
    rows is written (the pad of a padded pitch, the frame past the last).
    Whole tiles with a successor take the fixed-count store loop, float4 for
    a 16-B pitch ("padded", and "packed" when 3 n_sel is a multiple of 4) or
    single floats ("odd"), and frames past the trajectory in a 64-frame
    group rewrite its last row; the last tile of a segment takes the
    general form."""
    from rmsf_amd._lib import RMSF_XFORM_DOUBLES
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import motion_table
    n, nf, first, stride = shape
    eng = Engine()
    traj = torch.tensor(SY.frames(51, n, 0, nf, motion_table(52, nf)), device="cuda")
    sel_h = np.arange(first, n, stride)
    ns = len(sel_h)
    sel = eng.sel_tensor(sel_h)
    m = None
    if masses:
        m = torch.tensor(np.random.default_rng(53).uniform(1.0, 16.0, ns), device="cuda")
    dstride = {"packed": 3 * ns, "padded": (3 * ns + 3) // 4 * 4, "odd": 3 * ns + 5}[pitch]
    ref, info = eng.reference_setup(ns, frame_ptr=traj.data_ptr(), sel=sel, masses=m)
    work = eng.empty((eng.workspace_bytes(ns, nf) + 7) // 8)
    xf0 = eng.empty(nf, RMSF_XFORM_DOUBLES)
    xf1 = eng.empty(nf, RMSF_XFORM_DOUBLES)
    dense = torch.full((nf + 1, dstride), float("nan"), dtype=torch.float32, device="cuda")
    eng.superpose(traj.data_ptr(), 3 * n, nf, ns, sel, m, ref, info, xf0, work)
    eng.superpose(traj.data_ptr(), 3 * n, nf, ns, sel, m, ref, info, xf1, work, dense_out=dense.data_ptr(),
                  dense_stride=dstride)
    torch.cuda.synchronize()
    _same(xf1.cpu().numpy(), xf0.cpu().numpy(), "records")
    d = dense.cpu().numpy()
    want = traj.cpu().numpy()[:, sel_h].reshape(nf, 3 * ns)
    np.testing.assert_array_equal(d[:nf, :3 * ns].view(np.uint32), want.view(np.uint32))
    assert np.isnan(d[:nf, 3 * ns:]).all() and np.isnan(d[nf]).all()


@pytest.mark.parametrize("P", [1, 2])
def test_literal_shape_exact_gpus_list(lit, lit_traj, P):
    """The one-process form (gpus=[0] * P, the context ABI: rmsf_ctx_set_exact,
    sequential references / pushes, sweep-1 sums in rank order,
    rmsf_multi_chan_merge_exact) at RMSF.py's shape: the reference
    statements' P-rank run bit for bit."""
    from rmsf_amd import RMSF
    nf = 10
    r = RMSF(lit_traj[:nf], select=lit["sel"], masses=lit["masses"], align="average", exact=True,
             gpus=[0] * P).run().results
    for k, got in (("rmsf", r.rmsf), ("mean", r.mean), ("m2", r.sumsquares), ("average", r.average)):
        _same(np.reshape(got, lit[f"{k}_F{nf}_P{P}"].shape), lit[f"{k}_F{nf}_P{P}"], f"{k}, P={P}")


@pytest.mark.parametrize("align", ["frame0", "average"])
@pytest.mark.parametrize("P", [3, 4])
def test_exact_gpus_list_vs_oracle(align, P):
    """gpus=[0] * P (P contexts on the one device), aligned exact=True:
    equal to the oracle's P-rank restatement (rank-order sweep-1 sums,
    mpi4py's reduce tree) bit for bit, host input and HBM shards, with the
    per-frame rmsd."""
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    n, nf = 900, 23
    traj = SY.frames(51, n, 0, nf, motion_table(52, nf))
    sel = np.arange(2, n, 9)
    m = np.random.default_rng(53).uniform(1.0, 16.0, len(sel))
    want = O.rmsf_script(traj, sel, m, size=P, align=align)
    r = RMSF(traj, select=sel, masses=m, align=align, exact=True, gpus=[0] * P, collect_rmsd=True).run().results
    _same(r.rmsf, want["rmsf"], "rmsf")
    _same(r.mean, want["mean"], "mean")
    _same(r.sumsquares, want["m2"], "sumsquares")
    if align == "average":
        _same(r.average.reshape(-1, 3), want["average"], "average")
    assert r.rmsd.shape == (nf,)


def test_context_exact_aligned_push():
    """The torch-free context boundary: set_exact, the frame-0 reference,
    RMSF_PUSH_ALIGN_SUM, the average reference, RMSF_PUSH_ALIGN_WELFORD in
    three chunks (k continued) -- RMSF.py's one-rank statements bit for bit;
    a reference set before set_exact is refused by an exact aligned push."""
    from rmsf_amd import RmsfError
    from rmsf_amd.context import PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, Context
    from rmsf_amd.synth import motion_table
    n, nf = 1200, 31
    traj = SY.frames(61, n, 0, nf, motion_table(62, nf))
    sel = np.sort(np.random.default_rng(63).choice(n, 150, replace=False))
    m = np.full(len(sel), 12.011)
    want = O.rmsf_script(traj, sel, m, size=1, align="average")
    with Context(n, sel=sel, masses=m) as c:
        c.set_reference_frame(traj[0])
        c.set_exact(True, m)
        with pytest.raises(RmsfError):
            c.push(traj[:2], PUSH_ALIGN_SUM)
        c.set_reference_frame(traj[0])
        c.push(traj, PUSH_ALIGN_SUM)
        c.set_reference_average()
        for a, b in ((0, 10), (10, 11), (11, nf)):
            c.push(traj[a:b], PUSH_ALIGN_WELFORD)
        n_, mean, m2 = c.partial()
        assert n_ == nf
        _same(c.average().reshape(-1, 3), want["average"], "average")
        _same(mean.reshape(-1, 3), want["mean"], "mean")
        _same(m2.reshape(-1, 3), want["m2"], "sumsquares")
        _same(c.rmsf(), want["rmsf"], "rmsf")
