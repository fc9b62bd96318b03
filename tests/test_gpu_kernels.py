"""GPU tier, kernel level: every HIP kernel against the oracle through the C ABI.

Tolerances: integer/index work and the synthetic generator are bit-exact;
floating point follows the north star's 1e-6 A absolute bound on RMSF and
tighter bounds on intermediate f64 quantities (stated per assertion)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from rmsf_amd.engine import Engine
    return Engine()


def _sync():
    torch.cuda.synchronize()


def test_synth_bit_exact(eng):
    from rmsf_amd.synth import generate, motion_table
    d = np.load(os.path.join(GOLDEN, "synth_slice.npz"))
    g = generate(eng, 100, 0, 4, seed=5)
    gm = generate(eng, 100, 0, 4, seed=5, motion=d["motion"])
    _sync()
    np.testing.assert_array_equal(g.cpu().numpy(), d["frames"])
    np.testing.assert_array_equal(gm.cpu().numpy(), d["frames_motion"])
    # a large, odd-shaped slice deep into a big trajectory
    mt = motion_table(1, 5000)
    big = generate(eng, 1001, 4990, 10, seed=123, motion=mt)
    _sync()
    np.testing.assert_array_equal(big.cpu().numpy()[3:7, 200:400], SY.frames(123, 1001, 4993, 4, mt, np.arange(200, 400)))


def test_qcp_known_answer_device(eng):
    from rmsf_amd import CalcRMSDRotationalMatrix
    d = np.load(os.path.join(GOLDEN, "qcp_kat.npz"))
    ref = d["ref"] - d["ref"].mean(0)
    mob = d["mob"] - d["mob"].mean(0)
    rot = np.zeros(9)
    rmsd = CalcRMSDRotationalMatrix(ref, mob, 7, rot, None)
    assert rmsd == pytest.approx(0.7191064509622, abs=1e-12)
    np.testing.assert_allclose(rot.reshape(3, 3), d["rot"], atol=1e-7)
    with pytest.raises(ValueError):
        CalcRMSDRotationalMatrix(ref.astype(np.float32), mob, 7, rot, None)
    w = np.random.default_rng(0).uniform(0.5, 2, 7)
    rot_w = np.zeros(9)
    r_w = CalcRMSDRotationalMatrix(ref, mob, 7, rot_w, w)
    rot_o = np.zeros(9)
    r_o = O.CalcRMSDRotationalMatrix(ref, mob, 7, rot_o, w)
    assert r_w == pytest.approx(r_o, abs=1e-12)
    np.testing.assert_allclose(rot_w, rot_o, atol=1e-12)


def test_qcp_batch_vs_oracle(eng):
    rng = np.random.default_rng(5)
    As, E0s, Ns, exp = [], [], [], []
    for i in range(300):
        n = int(rng.integers(3, 200))
        ref = rng.normal(size=(n, 3)) * 10
        mob = ref @ O.kabsch(rng.normal(size=(3, 3)), rng.normal(size=(3, 3))) + rng.normal(size=(n, 3))
        ref -= ref.mean(0)
        mob -= mob.mean(0)
        A, E0 = O.inner_product(ref, mob)
        As.append(A)
        E0s.append(E0)
        Ns.append(n)
        exp.append(O.fast_calc_rmsd_and_rotation(A, E0, float(n)))
    dev = lambda a: torch.tensor(np.asarray(a, dtype=np.float64), device=eng.device)
    rot, rmsd = eng.qcp_batch(dev(As), dev(E0s), dev(Ns))
    _sync()
    np.testing.assert_allclose(rot.cpu().numpy(), np.array([e[0] for e in exp]), atol=1e-13)
    np.testing.assert_allclose(rmsd.cpu().numpy(), np.array([e[1] for e in exp]), atol=1e-11)


@pytest.mark.parametrize("masses", [False, True])
@pytest.mark.parametrize("gather", [False, True])
def test_reference_setup(eng, masses, gather):
    rng = np.random.default_rng(2)
    frame = SY.frames(3, 500, 7, 1)[0]
    sel = np.sort(rng.choice(500, 120, replace=False)) if gather else np.arange(500)
    m = rng.uniform(1, 16, len(sel)) if masses else None
    fdev = torch.tensor(frame, device=eng.device)
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    mdev = torch.tensor(m, device=eng.device) if masses else None
    ref, info = eng.reference_setup(len(sel), frame_ptr=fdev.data_ptr(), sel=sdev, masses=mdev)
    _sync()
    com, rc = O.centred_reference(frame[sel], m)
    np.testing.assert_allclose(info.cpu().numpy()[:3], com, rtol=0, atol=1e-12)
    np.testing.assert_allclose(ref.cpu().numpy(), rc, rtol=0, atol=1e-12)
    # from a float64 average
    avg = torch.tensor(rc + 3.0, device=eng.device).reshape(-1)
    ref2, info2 = eng.reference_setup(len(sel), avg=avg, masses=mdev)
    _sync()
    com2, rc2 = O.centred_reference(rc + 3.0, m)
    np.testing.assert_allclose(ref2.cpu().numpy(), rc2, atol=1e-12)


@pytest.mark.parametrize("n_sel", [1, 214, 1024, 1025])
def test_reference_setup_one_launch_bitwise(eng, n_sel):
    """Up to 1,024 selected atoms the reference setup is one launch
    (k_ref_setup1); its record and centred reference are bit-identical to the
    three launches it replaces (k_ref_com, k_ref_center, k_ref_finish), for
    frames and averages, gathered or not, with and without masses."""
    import ctypes

    L = eng.lib
    f3 = L.rmsf_internal_reference_setup3
    f3.restype = ctypes.c_int
    f3.argtypes = L.rmsf_reference_setup.argtypes
    rng = np.random.default_rng(n_sel)
    n_atoms = n_sel + 300
    frame = torch.tensor(rng.normal(0, 20, (n_atoms, 3)).astype(np.float32), device=eng.device)
    sel = torch.tensor(np.sort(rng.choice(n_atoms, n_sel, replace=False)).astype(np.int32), device=eng.device)
    avg = torch.tensor(rng.normal(5, 20, 3 * n_sel), device=eng.device)
    masses = torch.tensor(rng.uniform(1, 16, n_sel), device=eng.device)
    for src in ("frame", "frame_gather", "avg"):
        for m in (None, masses):
            outs = []
            for fn in (L.rmsf_reference_setup, f3):
                ref, info = eng.empty(n_sel, 3), eng.empty(16 + 2 * 4 * 256)
                info.fill_(7.0)
                fp = frame.data_ptr() if src != "avg" else None
                ap = avg.data_ptr() if src == "avg" else None
                sp = sel.data_ptr() if src == "frame_gather" else None
                mp = m.data_ptr() if m is not None else None
                assert fn(fp, ap, n_sel, sp, mp, ref.data_ptr(), info.data_ptr(), eng.stream) == 0
                outs.append((ref, info[:16].clone()))
            _sync()
            for a, b in zip(outs[0], outs[1]):
                assert torch.equal(a.view(torch.int64), b.view(torch.int64)), (src, m is not None)


@pytest.mark.parametrize("n_sel", [1, 214, 1024, 1025, 5000])
def test_reference_setup_mean_bitwise(eng, n_sel):
    """rmsf_reference_setup_mean (RMSF.py:111 + 113-118; one launch up to
    1,024 atoms) writes the average and the reference bit for bit as
    rmsf_divide + rmsf_reference_setup(avg) do."""
    rng = np.random.default_rng(n_sel + 1)
    total = torch.tensor(rng.normal(0, 2000, 3 * n_sel), device=eng.device)
    masses = torch.tensor(rng.uniform(1, 16, n_sel), device=eng.device)
    for m in (None, masses):
        avg, ref, info = eng.reference_setup_mean(total, 98.0, n_sel, m)
        avg2 = eng.empty(3 * n_sel)
        eng.divide(total, 98.0, avg2)
        ref2, info2 = eng.reference_setup(n_sel, avg=avg2, masses=m)
        _sync()
        for a, b in ((avg, avg2), (ref, ref2), (info[:16], info2[:16])):
            assert torch.equal(a.view(torch.int64), b.view(torch.int64)), m is not None


@pytest.mark.parametrize("gather", [False, True])
def test_superpose_vs_oracle(eng, gather):
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = 5000 if not gather else 9000, 37
    mt = motion_table(4, nf)
    traj = generate(eng, n_atoms, 0, nf, seed=9, motion=mt)
    sel = np.sort(np.random.default_rng(1).choice(n_atoms, 4500, replace=False)) if gather else np.arange(n_atoms)
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    ref, info = eng.reference_setup(len(sel), frame_ptr=traj.data_ptr(), sel=sdev)
    xf = eng.empty(nf, 16)
    work = eng.empty(eng.workspace_bytes(len(sel), nf) // 8 + 1)
    eng.superpose(traj.data_ptr(), 3 * n_atoms, nf, len(sel), sdev, None, ref, info, xf, work)
    _sync()
    xf = xf.cpu().numpy()
    host = traj.cpu().numpy()
    ref_com, ref_c = O.centred_reference(host[0][sel])
    for f in range(nf):
        p = host[f][sel]
        com = O.center_of_mass(p)
        R = O.get_rotation_matrix(ref_c, p.astype(np.float64) - com, len(sel))
        np.testing.assert_allclose(xf[f, 9:12], com, atol=1e-9)
        np.testing.assert_allclose(xf[f, :9].reshape(3, 3), R, atol=1e-10)


@pytest.mark.parametrize("n_sel,nf,splits", [(4096, 1000, None), (4096, 1000, 7), (1001, 333, None),
                                              (3, 5, 1), (100_000, 64, None)])
def test_welford_noalign(eng, n_sel, nf, splits):
    from rmsf_amd.synth import generate
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    traj = generate(eng, n_sel, 0, nf, seed=21)
    s = splits or eng.splits(n_sel, nf, False)
    mp = eng.empty(s, 3 * n_sel)
    qp = eng.empty(s, 3 * n_sel)
    eng.accumulate(traj.data_ptr(), 3 * n_sel, nf, n_sel, None, None, None, RMSF_MODE_WELFORD, s, mp, qp)
    mean, m2 = eng.empty(3 * n_sel), eng.empty(3 * n_sel)
    eng.chan_merge(mp, qp, eng.split_counts(nf, s), 3 * n_sel, mean, m2)
    rmsf = eng.empty(n_sel)
    eng.finalize(m2, n_sel, nf, rmsf)
    _sync()
    host = traj.cpu().numpy()
    x = host.astype(np.float64)
    np.testing.assert_allclose(mean.cpu().numpy().reshape(-1, 3), x.mean(0), rtol=0, atol=1e-10)
    np.testing.assert_allclose(rmsf.cpu().numpy(), O.rmsf_two_pass(host), rtol=0, atol=1e-9)
    if n_sel == 4096 and nf == 1000:
        d = np.load(os.path.join(GOLDEN, "noalign_4096.npz"))
        np.testing.assert_allclose(rmsf.cpu().numpy(), d["rmsf_P1"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("n_sel,nf,groups,gather", [
    (4096, 1000, 0, False), (4096, 1000, 1, False), (4096, 1000, 3, False), (1001, 333, 0, False),
    (1001, 333, 7, True), (3, 5, 0, False), (3, 5, 2, True), (300, 9000, 1, False), (300, 9000, 5, True),
    (2048, 700, 3000, False), (100_000, 64, 0, False), (257, 4097, 2, False),
    (300_000, 64, 0, False), (300_000, 33, 0, False), (250_000, 50, 0, True)])
def test_balanced_welford_and_sum(eng, n_sel, nf, groups, gather):
    """Balanced grid (rmsf_accumulate_balanced + rmsf_fold_balanced): float4
    and atom-per-lane layouts, forced workgroup counts (1 = one workgroup
    walks every chunk; 9000 frames cut segments at RMSF_MAX_SPLIT_FRAMES;
    3000 > the chunk-frame count clamps; 250k-300k atoms: more chunks than
    workgroups, chunk-aligned ranges), and a running fold over two batches,
    against the f64 two-pass variance and the f64 sum."""
    from rmsf_amd.synth import generate
    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_MODE_WELFORD
    n_atoms = n_sel + 17 if gather else n_sel
    traj = generate(eng, n_atoms, 0, nf, seed=22)
    sel = np.sort(np.random.default_rng(3).choice(n_atoms, n_sel, replace=False)) if gather else None
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    host = traj.cpu().numpy()
    x = (host[:, sel] if gather else host).astype(np.float64)
    cut = nf // 3
    mean, m2, s = eng.empty(3 * n_sel), eng.empty(3 * n_sel), eng.empty(3 * n_sel)
    acc = 0
    for f0, f1 in ((0, cut), (cut, nf)):
        if f1 <= f0:
            continue
        n = f1 - f0
        work = eng.empty(eng.balanced_workspace_bytes(n_sel, n, groups) // 8 + 2)
        ptr = traj.data_ptr() + f0 * 3 * n_atoms * 4
        eng.accumulate_balanced(ptr, 3 * n_atoms, n, n_sel, sdev, None, None, RMSF_MODE_WELFORD, work, groups)
        eng.fold_balanced(work, 3 * n_sel, RMSF_MODE_WELFORD, acc, mean, m2)
        eng.accumulate_balanced(ptr, 3 * n_atoms, n, n_sel, sdev, None, None, RMSF_MODE_SUM, work, groups)
        eng.fold_balanced(work, 3 * n_sel, RMSF_MODE_SUM, acc, s, None)
        acc += n
    rmsf = eng.empty(n_sel)
    eng.finalize(m2, n_sel, nf, rmsf)
    _sync()
    np.testing.assert_allclose(mean.cpu().numpy().reshape(-1, 3), x.mean(0), rtol=0, atol=1e-10)
    np.testing.assert_allclose(s.cpu().numpy().reshape(-1, 3), x.sum(0), rtol=1e-13, atol=1e-9)
    np.testing.assert_allclose(rmsf.cpu().numpy(), O.rmsf_two_pass(x), rtol=0, atol=1e-9)


@pytest.mark.parametrize("n_sel,nf,groups,gather", [
    (4096, 1000, 0, False), (1001, 333, 7, True), (3, 5, 0, False), (3, 5, 2, True), (257, 4097, 2, False),
    (300, 9000, 0, True), (1000, 1, 0, False), (1000, 2, 0, False), (5000, 3, 1, False), (70_000, 40, 0, False)])
def test_balanced_aligned_vs_split_grid(eng, n_sel, nf, groups, gather):
    """The aligned accumulate on the balanced grid -- k_accum_split_sk: each
    segment's frames split over Q sub-blocks that share one shift (1-3 frame
    segments leave sub-blocks empty) -- against the split grid's one-atom-per-
    lane kernel (k_accum_atoms) on the same device transforms: the f32
    transformed coordinates are the same values, only the f64 summation order
    differs (1e-10).  Both against RMSF.py:133-138 restated in numpy with the
    device's R / COM and the three f32 rounding points (1e-6 A, the north
    star's bound: an FMA-order flip moves one coordinate by one f32 ulp)."""
    from rmsf_amd.synth import generate, motion_table
    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_MODE_WELFORD
    n_atoms = n_sel + 11 if gather else n_sel
    traj = generate(eng, n_atoms, 0, nf, seed=31, motion=motion_table(2, nf))
    sel = np.sort(np.random.default_rng(4).choice(n_atoms, n_sel, replace=False)) if gather else np.arange(n_sel)
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    ref, info = eng.reference_setup(n_sel, frame_ptr=traj.data_ptr(), sel=sdev)
    xf = eng.empty(nf, 16)
    sw = eng.empty(eng.workspace_bytes(n_sel, nf) // 8 + 1)
    eng.superpose(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, None, ref, info, xf, sw)
    nc = 3 * n_sel
    # balanced grid, two batches folded in order
    mean, m2, s = eng.empty(nc), eng.empty(nc), eng.empty(nc)
    acc, cut = 0, nf // 3
    for f0, f1 in ((0, cut), (cut, nf)):
        if f1 <= f0:
            continue
        n = f1 - f0
        work = eng.empty(eng.balanced_workspace_bytes(n_sel, n, groups) // 8 + 2)
        ptr = traj.data_ptr() + f0 * 3 * n_atoms * 4
        eng.accumulate_balanced(ptr, 3 * n_atoms, n, n_sel, sdev, xf[f0:], info, RMSF_MODE_WELFORD, work, groups)
        eng.fold_balanced(work, nc, RMSF_MODE_WELFORD, acc, mean, m2)
        eng.accumulate_balanced(ptr, 3 * n_atoms, n, n_sel, sdev, xf[f0:], info, RMSF_MODE_SUM, work, groups)
        eng.fold_balanced(work, nc, RMSF_MODE_SUM, acc, s, None)
        acc += n
    # split grid
    k = eng.splits(n_sel, nf, True)
    mp, qp, sp = eng.empty(k, nc), eng.empty(k, nc), eng.empty(k, nc)
    eng.accumulate(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, xf, info, RMSF_MODE_WELFORD, k, mp, qp)
    mean_s, m2_s, s_s = eng.empty(nc), eng.empty(nc), eng.empty(nc)
    eng.chan_merge(mp, qp, eng.split_counts(nf, k), nc, mean_s, m2_s)
    eng.accumulate(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, xf, info, RMSF_MODE_SUM, k, sp, None)
    eng.sum_splits(sp, k, nc, s_s)
    _sync()
    M, Q2, S = mean.cpu().numpy(), m2.cpu().numpy(), s.cpu().numpy()
    np.testing.assert_allclose(M, mean_s.cpu().numpy(), rtol=0, atol=1e-10)
    np.testing.assert_allclose(S, s_s.cpu().numpy(), rtol=1e-13, atol=1e-9)
    np.testing.assert_allclose(Q2 / nf, m2_s.cpu().numpy() / nf, rtol=0, atol=1e-10)
    # RMSF.py:133-138 with the device's transforms
    X, I = xf.cpu().numpy(), info.cpu().numpy()
    host = traj.cpu().numpy()[:, sel].astype(np.float64)
    al = np.empty_like(host)
    for f in range(nf):
        p = (host[f] - X[f, 9:12]).astype(np.float32).astype(np.float64)
        p = (p @ X[f, :9].reshape(3, 3)).astype(np.float32).astype(np.float64)
        al[f] = (p + I[:3]).astype(np.float32)
    np.testing.assert_allclose(M.reshape(-1, 3), al.mean(0), rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.sqrt(Q2.reshape(-1, 3).sum(1) / nf), O.rmsf_two_pass(al), rtol=0, atol=1e-6)


@pytest.mark.parametrize("n_sel,nf,gather", [(214, 98, True), (1, 5, False), (3000, 700, False),
                                             (20000, 64, True)])
def test_fold_finalize_bitwise(eng, n_sel, nf, gather):
    """rmsf_fold_balanced_finalize (the aligned sweep's last fold + the
    RMSF.py:146 finalise, one launch) writes mean, M2 and RMSF bit for bit as
    rmsf_fold_balanced + rmsf_finalize, after a first batch (acc_n > 0) too;
    on a flat plan (unaligned contiguous selection) the call is refused with
    RMSF_EINVAL instead of writing NaN."""
    from rmsf_amd.synth import generate, motion_table
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    n_atoms = n_sel + 5 if gather else n_sel
    traj = generate(eng, n_atoms, 0, nf, seed=5, motion=motion_table(3, nf))
    sel = np.sort(np.random.default_rng(6).choice(n_atoms, n_sel, replace=False)) if gather else None
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    ref, info = eng.reference_setup(n_sel, frame_ptr=traj.data_ptr(), sel=sdev)
    xf = eng.empty(nf, 16)
    sw = eng.empty(eng.workspace_bytes(n_sel, nf) // 8 + 1)
    eng.superpose(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, None, ref, info, xf, sw)
    nc = 3 * n_sel
    out = []
    for fused in (False, True):
        mean, m2, r = eng.empty(nc), eng.empty(nc), eng.empty(n_sel)
        acc, cut = 0, nf // 2
        for f0, f1 in ((0, cut), (cut, nf)):
            if f1 <= f0:
                continue
            n = f1 - f0
            work = eng.empty(eng.balanced_workspace_bytes(n_sel, n) // 8 + 2)
            ptr = traj.data_ptr() + f0 * 3 * n_atoms * 4
            eng.accumulate_balanced(ptr, 3 * n_atoms, n, n_sel, sdev, xf[f0:], info, RMSF_MODE_WELFORD, work)
            if fused and f1 == nf:
                eng.fold_balanced_finalize(work, nc, acc, mean, m2, nf, r)
            else:
                eng.fold_balanced(work, nc, RMSF_MODE_WELFORD, acc, mean, m2)
            acc += n
        if not fused:
            eng.finalize(m2, n_sel, nf, r)
        out.append((mean, m2, r))
    _sync()
    for a, b in zip(*out):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    if not gather and n_sel % 4 == 0:  # the flat plan: an atom spans two lanes -> the second launch
        work = eng.empty(eng.balanced_workspace_bytes(n_sel, nf) // 8 + 2)
        eng.accumulate_balanced(traj.data_ptr(), 3 * n_atoms, nf, n_sel, None, None, None, RMSF_MODE_WELFORD, work)
        mean, m2, r = eng.empty(nc), eng.empty(nc), eng.zeros(n_sel)
        eng.fold_balanced_finalize(work, nc, 0, mean, m2, nf, r)
        want = eng.empty(n_sel)
        eng.finalize(m2, n_sel, nf, want)
        _sync()
        assert torch.equal(r.view(torch.int64), want.view(torch.int64))


def _plan_workspace_case(eng, flat: bool, work=None):
    """One balanced accumulate of a small unaligned batch (flat plan: a
    contiguous selection of 4k atoms; atom plan: a gathered selection) into
    ``work``, then rmsf_fold_balanced_finalize; returns (rmsf, reference
    finalize) tensors."""
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    from rmsf_amd.synth import generate
    n_sel, nf = 64, 9
    traj = generate(eng, n_sel + 3, 0, nf, seed=17)
    sel = None if flat else eng.sel_tensor(np.arange(2, n_sel + 2))
    need = eng.balanced_workspace_bytes(n_sel, nf) // 8 + 2
    if work is None or work.numel() < need:
        work = eng.empty(need)
    fs = 3 * (n_sel + 3)
    if flat:   # contiguous rows of exactly n_sel atoms: the flat float4 plan
        traj = generate(eng, n_sel, 0, nf, seed=17)
        fs = 3 * n_sel
    eng.accumulate_balanced(traj.data_ptr(), fs, nf, n_sel, sel, None, None, RMSF_MODE_WELFORD, work)
    mean, m2, r = eng.empty(3 * n_sel), eng.empty(3 * n_sel), eng.zeros(n_sel)
    eng.fold_balanced_finalize(work, 3 * n_sel, 0, mean, m2, nf, r)
    want = eng.empty(n_sel)
    eng.finalize(m2, n_sel, nf, want)
    return r, want, work


def test_fold_finalize_plan_from_workspace_header(eng):
    """ADVICE r4 / VERDICT r4 item 4: the plan fold_balanced_finalize acts on
    is read from the workspace's own header on the device, not from a host
    record of allocations -- after more than 4,096 workspaces, and when a
    freed workspace's memory is reused by the other plan kind (both orders),
    flat and atom plans alike finalise bit-identically to rmsf_finalize."""
    outs = []
    keep = []
    for i in range(4100):   # many live workspaces (the old host map held 4,096)
        keep.append(eng.empty(8))
    for flat in (True, False):
        outs.append(_plan_workspace_case(eng, flat)[:2])
    del keep
    # one buffer, reused: atom plan, then flat, then atom again
    r1, w1, work = _plan_workspace_case(eng, False)
    r2, w2, work = _plan_workspace_case(eng, True, work)
    r3, w3, work = _plan_workspace_case(eng, False, work)
    outs += [(r1, w1), (r2, w2), (r3, w3)]
    # a freed workspace whose address the allocator hands out again
    ptr = work.data_ptr()
    del work
    torch.cuda.synchronize()
    r4, w4, work = _plan_workspace_case(eng, True)
    outs.append((r4, w4))
    _sync()
    for r, w in outs:
        assert torch.isfinite(r).all()
        assert torch.equal(r.view(torch.int64), w.view(torch.int64))
    print(f"reused address: {work.data_ptr() == ptr}")


def test_balanced_bad_arguments(eng):
    from rmsf_amd import RmsfError
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    x = eng.empty(10, 3, dtype=torch.float32)
    small = eng.empty(4)
    with pytest.raises(RmsfError, match="workspace too small"):
        eng.accumulate_balanced(x.data_ptr(), 3, 10, 1, None, None, None, RMSF_MODE_WELFORD, small)
    with pytest.raises(RmsfError, match="bad arguments"):
        eng.accumulate_balanced(x.data_ptr(), 3, 0, 1, None, None, None, RMSF_MODE_WELFORD, small)


def test_chan_merge_kernel_many_groups(eng):
    """>128 partials exercise the grouped launches; counts with empties."""
    rng = np.random.default_rng(0)
    counts = [int(c) for c in rng.integers(0, 5, 300)]
    counts[0] = 0
    n = 33
    data = [rng.normal(size=(c, n)) for c in counts]
    mp = np.stack([d.mean(0) if len(d) else np.zeros(n) for d in data])
    qp = np.stack([((d - d.mean(0)) ** 2).sum(0) if len(d) else np.zeros(n) for d in data])
    mean, m2 = eng.empty(n), eng.empty(n)
    eng.chan_merge(torch.tensor(mp, device=eng.device), torch.tensor(qp, device=eng.device), counts, n, mean, m2)
    _sync()
    allx = np.concatenate([d for d in data if len(d)])
    np.testing.assert_allclose(mean.cpu().numpy(), allx.mean(0), atol=1e-12)
    np.testing.assert_allclose(m2.cpu().numpy(), ((allx - allx.mean(0)) ** 2).sum(0), rtol=1e-11)
    from rmsf_amd import RmsfEmptyError
    with pytest.raises(ZeroDivisionError):
        eng.chan_merge(torch.tensor(mp, device=eng.device), torch.tensor(qp, device=eng.device), [0] * 300, n,
                       mean, m2)
    assert issubclass(RmsfEmptyError, ZeroDivisionError)


@pytest.mark.parametrize("shift_kind", ["f64", "f64+off3", "f32"])
def test_chan_shift_merge_kernels(eng, shift_kind):
    """k_chan_shift_pack / k_chan_shift_finish: the one-all-reduce merge
    (parallel.global_chan_shifted) of P rank partials -- the packed sums
    added as the all-reduce would -- against the pooled mean / M2 / RMSF
    (RMSF.py:140-146) and against the two-collective Chan kernels; identical
    frames give exactly 0 when the shift is the data."""
    rng = np.random.default_rng(5)
    n_sel, counts = 211, [7, 0, 13, 1]
    n = 3 * n_sel
    base = rng.uniform(0, 100, n)
    data = [base + rng.normal(scale=1.5, size=(c, n)) for c in counts]
    mp = [d.mean(0) if len(d) else np.zeros(n) for d in data]
    qp = [((d - d.mean(0)) ** 2).sum(0) if len(d) else np.zeros(n) for d in data]
    nt = sum(counts)
    f0 = data[0][0].astype(np.float32)
    if shift_kind == "f32":
        shift, off3 = torch.tensor(f0, device=eng.device), None
    elif shift_kind == "f64":
        shift, off3 = torch.tensor(f0.astype(np.float64), device=eng.device), None
    else:
        com = f0.reshape(-1, 3).astype(np.float64).mean(0)
        shift = torch.tensor(f0.reshape(-1, 3) - com, device=eng.device).reshape(-1)
        off3 = torch.tensor(com, device=eng.device)
    t = torch.zeros(2 * n, dtype=torch.float64, device=eng.device)
    for m, q, c in zip(mp, qp, counts):
        tk = eng.empty(2 * n)
        eng.chan_shift_pack(torch.tensor(m, device=eng.device), torch.tensor(q, device=eng.device), shift, off3, c, tk)
        t += tk  # the all-reduce's sum
    mean, m2, rmsf = eng.empty(n), eng.empty(n), eng.empty(n_sel)
    eng.chan_shift_finish(t, shift, off3, n_sel, nt, mean, m2, rmsf)
    _sync()
    allx = np.concatenate([d for d in data if len(d)])
    q_all = ((allx - allx.mean(0)) ** 2).sum(0)
    np.testing.assert_allclose(mean.cpu().numpy(), allx.mean(0), rtol=0, atol=1e-12)
    np.testing.assert_allclose(m2.cpu().numpy(), q_all, rtol=1e-11)
    np.testing.assert_allclose(rmsf.cpu().numpy(), np.sqrt(q_all.reshape(-1, 3).sum(1) / nt), rtol=0, atol=1e-12)
    # identical frames about the same frame: exactly zero
    same = torch.tensor(np.tile(f0.astype(np.float64), 1), device=eng.device)
    tk = eng.empty(2 * n)
    eng.chan_shift_pack(same, torch.zeros(n, dtype=torch.float64, device=eng.device),
                        torch.tensor(f0, device=eng.device), None, 5, tk)
    eng.chan_shift_finish(tk, torch.tensor(f0, device=eng.device), None, n_sel, 5, mean, m2, rmsf)
    _sync()
    assert float(rmsf.abs().max()) == 0.0 and float(m2.abs().max()) == 0.0
    np.testing.assert_array_equal(mean.cpu().numpy(), f0.astype(np.float64))


def _segment_walks(work):
    """For every lane chunk of the balanced plan in ``work``: its segments'
    (partial slot, frame count) in frame order -- the walk k_fold_sk replays
    (sk_lo / sk_seg_len, segments cut at RMSF_MAX_SPLIT_FRAMES = 4096)."""
    h = work[:16].view(np.int64)
    lanes, C, nf, T, G, P, cpl, mode, S, cw = (int(v) for v in h[:10])

    def seg_len(lo, hi):
        return min(hi - lo, nf - lo % nf, 4096)

    walks = []
    for c in range(C):
        clo, chi = c * nf, c * nf + nf
        b = clo * G // T
        while b > 0 and T * b // G > clo:
            b -= 1
        while T * (b + 1) // G <= clo:
            b += 1
        lo, hi, slot = T * b // G, T * (b + 1) // G, b * P
        while lo < clo:
            lo += seg_len(lo, hi)
            slot += 1
        segs = []
        while True:
            if lo >= hi:
                b += 1
                if b >= G:
                    break
                lo, hi, slot = T * b // G, T * (b + 1) // G, b * P
            if lo >= chi:
                break
            n = seg_len(lo, hi)
            segs.append((slot, n))
            lo += n
            slot += 1
        walks.append(segs)
    return dict(G=G, P=P, cpl=cpl, cw=cw, slot_d=cw * cpl), walks


@pytest.mark.parametrize("n_sel,nf,groups,gather", [
    (4096, 9000, 0, False), (4096, 1000, 3, False), (1001, 333, 7, True), (257, 4097, 2, False),
    (300_000, 64, 0, False), (3, 5, 2, True)])
def test_fold_is_reference_chan_merge(eng, n_sel, nf, groups, gather):
    """k_fold_sk bit for bit against RMSF.py:36-41's own second_order_moments
    (the oracle's verbatim restatement, numpy) applied to the accumulate's
    segment partials in frame order, after a running state (acc_n > 0) too;
    the SUM fold against numpy's sequential sum.  Holds because the library
    is built without FP contraction (csrc/Makefile): the device evaluates the
    merge's expressions exactly as numpy does.  Flat and atom plans, segments
    cut at 4096 frames, forced workgroup counts, chunk-aligned ranges."""
    from rmsf_amd.synth import generate
    from rmsf_amd._lib import RMSF_MODE_SUM, RMSF_MODE_WELFORD
    n_atoms = n_sel + 5 if gather else n_sel
    traj = generate(eng, n_atoms, 0, nf, seed=41)
    sel = np.sort(np.random.default_rng(8).choice(n_atoms, n_sel, replace=False)) if gather else None
    sdev = torch.tensor(sel.astype(np.int32), device=eng.device) if gather else None
    nc = 3 * n_sel
    rng = np.random.default_rng(n_sel)
    acc_n = 7
    run_mean, run_m2 = rng.normal(40, 3, nc), rng.uniform(0, 5, nc)
    for mode in (RMSF_MODE_WELFORD, RMSF_MODE_SUM):
        work = eng.empty(eng.balanced_workspace_bytes(n_sel, nf, groups) // 8 + 2)
        eng.accumulate_balanced(traj.data_ptr(), 3 * n_atoms, nf, n_sel, sdev, None, None, mode, work, groups)
        outs = []
        for a_n in (0, acc_n):
            m0 = torch.tensor(run_mean, device=eng.device)
            m1 = torch.tensor(run_m2, device=eng.device) if mode == RMSF_MODE_WELFORD else None
            eng.fold_balanced(work, nc, mode, a_n, m0, m1)
            outs.append((m0, m1))
        _sync()
        wk = work.cpu().numpy()
        pl, walks = _segment_walks(wk)
        p0 = wk[16:]
        p1 = p0[pl["G"] * pl["P"] * pl["slot_d"]:]
        for (m0, m1), a_n in zip(outs, (0, acc_n)):
            got0 = m0.cpu().numpy()
            got1 = m1.cpu().numpy() if m1 is not None else None
            for c, segs in enumerate(walks):
                j0 = c * pl["slot_d"]
                j1 = min(j0 + pl["slot_d"], nc)
                if j0 >= nc:
                    break
                rows = [(n, p0[s * pl["slot_d"]:s * pl["slot_d"] + j1 - j0], p1[s * pl["slot_d"]:s * pl["slot_d"] + j1 - j0])
                        for s, n in segs]
                if mode == RMSF_MODE_WELFORD:
                    S = (a_n, run_mean[j0:j1], run_m2[j0:j1]) if a_n else (rows[0][0], rows[0][1], rows[0][2])
                    for n, mu, m2 in rows[0 if a_n else 1:]:
                        S = O.second_order_moments(S, (n, mu, m2))
                    want0, want1 = S[1], S[2]
                    np.testing.assert_array_equal(got1[j0:j1].view(np.uint64), np.asarray(want1).view(np.uint64),
                                                  err_msg=f"M2 chunk {c} acc_n {a_n}")
                else:
                    want0 = run_mean[j0:j1].copy() if a_n else np.zeros(j1 - j0)
                    for _, part, _ in rows:
                        want0 = want0 + part
                np.testing.assert_array_equal(got0[j0:j1].view(np.uint64), np.asarray(want0).view(np.uint64),
                                              err_msg=f"mode {mode} chunk {c} acc_n {a_n}")


@pytest.mark.parametrize("shift_kind", ["f64", "f64+off3", "f32"])
@pytest.mark.parametrize("n_sel,nf,groups", [(4096, 1000, 0), (1001, 333, 7), (3, 5, 2), (100_000, 64, 0),
                                            (300_000, 33, 0)])
def test_fold_balanced_shift_bitwise(eng, shift_kind, n_sel, nf, groups):
    """rmsf_fold_balanced_shift (the N > 1 pipeline's last fold) equals
    rmsf_fold_balanced + rmsf_chan_shift_pack bit for bit: the running result
    and the merge's T1/T2, over two batches (acc_n > 0 on the second)."""
    from rmsf_amd.synth import generate
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    traj = generate(eng, n_sel, 0, nf, seed=27)
    nc = 3 * n_sel
    f0 = traj[0].reshape(-1)
    if shift_kind == "f32":
        shift, off3 = f0.clone(), None
    elif shift_kind == "f64":
        shift, off3 = f0.double(), None
    else:
        com = f0.double().reshape(-1, 3).mean(0)
        shift, off3 = (f0.double().reshape(-1, 3) - com).reshape(-1), com.contiguous()
    outs = []
    for fused in (False, True):
        mean, m2 = eng.empty(nc), eng.empty(nc)
        t = torch.full((2 * nc,), float("nan"), dtype=torch.float64, device=eng.device)
        acc, cut = 0, nf // 3
        for f0_, f1_ in ((0, cut), (cut, nf)):
            if f1_ <= f0_:
                continue
            n = f1_ - f0_
            work = eng.empty(eng.balanced_workspace_bytes(n_sel, n, groups) // 8 + 2)
            ptr = traj.data_ptr() + f0_ * 3 * n_sel * 4
            eng.accumulate_balanced(ptr, 3 * n_sel, n, n_sel, None, None, None, RMSF_MODE_WELFORD, work, groups)
            if fused and f1_ == nf:
                eng.fold_balanced_shift(work, nc, acc, mean, m2, shift, off3, t)
            else:
                eng.fold_balanced(work, nc, RMSF_MODE_WELFORD, acc, mean, m2)
            acc += n
        if not fused:
            eng.chan_shift_pack(mean, m2, shift, off3, float(acc), t)
        _sync()
        outs.append([x.cpu().numpy() for x in (mean, m2, t)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    assert np.isfinite(outs[1][2]).all()


def test_second_order_moments_api(eng):
    from rmsf_amd import second_order_moments
    rng = np.random.default_rng(1)
    a, b = rng.normal(size=(7, 10, 3)), rng.normal(size=(4, 10, 3)) + 1
    S1 = [7, a.mean(0), ((a - a.mean(0)) ** 2).sum(0)]
    S2 = [4, b.mean(0), ((b - b.mean(0)) ** 2).sum(0)]
    T, mu, M = second_order_moments(S1, S2)
    Te, mue, Me = O.second_order_moments(S1, S2)
    assert T == Te
    np.testing.assert_allclose(mu, mue, atol=1e-14)
    np.testing.assert_allclose(M, Me, rtol=1e-13)
    with pytest.raises(ZeroDivisionError):
        second_order_moments([0, np.zeros((10, 3)), np.zeros((10, 3))], [0, np.zeros((10, 3)), np.zeros((10, 3))])


def test_error_paths(eng):
    from rmsf_amd import RmsfError
    from rmsf_amd._lib import RMSF_MODE_WELFORD
    x = eng.empty(10, 3, dtype=torch.float32)
    out = eng.empty(30)
    with pytest.raises(RmsfError, match="bad arguments"):
        eng.accumulate(x.data_ptr(), 3, 10, 0, None, None, None, RMSF_MODE_WELFORD, 1, out, out)
    with pytest.raises(RmsfError, match="RMSF_MAX_SPLIT_FRAMES"):
        eng.accumulate(x.data_ptr(), 30, 10000, 10, None, None, None, RMSF_MODE_WELFORD, 1, out, out)
