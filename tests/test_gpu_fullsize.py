"""GPU tier at BASELINE.json's full sizes, checked through size-independent
properties: sampled atoms regenerated bit-exactly on the CPU (counter-based
generator) against an independent two-pass variance, the analytic
sqrt(3)*sigma of the generator, invariance under the frame-tile split; for
the aligned sweeps, the device's per-frame rotation and mobile COM pinned on
sampled frames against the CPU QCP over the whole selection, and 48 sampled
atoms' statistics rebuilt from RMSF.py's per-frame loop with those
transforms (1e-6 A).

  C2  100k atoms x 20k frames, no alignment           (24 GB in HBM)
  C3  100k atoms x 20k frames, QCP to frame 0         (24 GB)
  C4  1M atoms x 2.5k frames (one GPU's share at N=8) (30 GB)
  RMSF.py's two sweeps (align="average") at C3's size
"""
import numpy as np
import pytest
import torch

from oracle import rmsf_oracle as O
from oracle import synth as SY

pytestmark = pytest.mark.gpu
TOL = 1e-6  # Angstrom, absolute (north star)


def _release(*ts):
    for t in ts:
        del t
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n_atoms,nf", [(100_000, 20_000), (1_000_000, 2_500)], ids=["C2", "C4share"])
def test_full_size_unaligned(n_atoms, nf):
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate
    traj = generate(Engine(), n_atoms, 0, nf, seed=0)
    r = RMSF(traj).run().results
    assert r.n_frames == nf and r.rmsf.shape == (n_atoms,)
    atoms = np.sort(np.random.default_rng(n_atoms).choice(n_atoms, 48, replace=False))
    host = SY.frames(0, n_atoms, 0, nf, atoms=atoms)
    np.testing.assert_allclose(r.rmsf[atoms], O.rmsf_two_pass(host), rtol=0, atol=1e-9)
    np.testing.assert_allclose(r.mean[atoms], host.astype(np.float64).mean(axis=0), rtol=0, atol=1e-9)
    # analytic: the generator's per-atom spread is sqrt(3) sigma
    np.testing.assert_allclose(r.rmsf, SY.expected_rmsf(0, np.arange(n_atoms)), rtol=0.05)
    # the frame-tile split is an internal choice: 3 tiles vs the default
    s = RMSF(traj, n_splits=3).run().results
    np.testing.assert_allclose(s.rmsf, r.rmsf, rtol=0, atol=1e-12)
    # exact=True: RMSF.py:137-138's recurrence over all nf frames, bit for
    # bit on the sampled atoms (the oracle's rank_sweep2 on their columns)
    e = RMSF(traj, exact=True).run().results
    S = O.rank_sweep2(host, np.arange(48), None, 0, nf)
    for got, want in ((e.mean[atoms], S[1]), (e.sumsquares[atoms], S[2]),
                      (e.rmsf[atoms], np.sqrt(S[2].sum(axis=1) / nf))):
        np.testing.assert_array_equal(got.view(np.uint64), np.ascontiguousarray(want).view(np.uint64))
    np.testing.assert_allclose(e.rmsf, r.rmsf, rtol=0, atol=1e-11)
    _release(traj)


N_FULL, NF_FULL = 100_000, 20_000
SAMPLE_FRAMES = (0, 1, 2, 777, 5_000, 12_345, NF_FULL - 2, NF_FULL - 1)


def _sampled_atoms(n_atoms):
    return np.sort(np.random.default_rng(n_atoms + 3).choice(n_atoms, 48, replace=False))


def _check_records(traj, T, ref_full_f64, frames=SAMPLE_FRAMES):
    """Device transform records of sampled frames against the CPU
    restatement of RMSF.py:94-97 + 48-51 on the whole selection: mobile COM
    and the QCP rotation to the centred reference."""
    ref_com, ref_c = O.centred_reference(ref_full_f64)
    dR = dC = 0.0
    for f in frames:
        mob = traj[f].cpu().numpy()
        com = O.center_of_mass(mob).astype(np.float64)
        R = O.get_rotation_matrix(ref_c, mob.astype(np.float64) - com, len(mob))
        np.testing.assert_allclose(T[f, 9:12], com, rtol=0, atol=1e-9, err_msg=f"COM of frame {f}")
        np.testing.assert_allclose(T[f, :9], R.reshape(-1), rtol=0, atol=1e-9, err_msg=f"R of frame {f}")
        dR = max(dR, np.abs(T[f, :9] - R.reshape(-1)).max())
        dC = max(dC, np.abs(T[f, 9:12] - com).max())
    print(f"\n  sampled frames {list(frames)}: max|dR| {dR:.2e}, max|dCOM| {dC:.2e} A")
    return ref_com


def _aligned_rows(rows, T, ref_com):
    """RMSF.py:99-101 / 133-135 on the sampled rows of every frame, with the
    device's per-frame rotation and mobile COM (pinned by _check_records)."""
    out = np.empty_like(rows)
    for f in range(rows.shape[0]):
        p = rows[f].copy()
        O.apply_transform_(p, T[f, :9].reshape(3, 3), T[f, 9:12], ref_com)
        out[f] = p
    return out


def _welford_rmsf(aligned):
    """RMSF.py:136-138 + 146 over the aligned rows (one rank)."""
    S = O.rank_sweep2(aligned, np.arange(aligned.shape[1]), None, 0, aligned.shape[0])
    return S[1], np.sqrt(S[2].sum(axis=1) / S[0])


def test_full_size_aligned_c3():
    """C3 (100k x 20k, QCP to frame 0) pinned at full size: device R/COM of
    8 sampled frames against the CPU QCP on all 100k atoms (1e-9), then 48
    sampled atoms' mean and RMSF rebuilt through RMSF.py:133-138 with the
    device's per-frame R/COM over all 20k frames, within 1e-6 A."""
    import torch as _t
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = N_FULL, NF_FULL
    traj = generate(Engine(), n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    r = RMSF(traj, align="frame0", collect_rmsd=True, collect_transforms=True).run().results
    T = r.transforms
    assert T.shape == (nf, 16) and r.rmsd.shape == (nf,) and r.rmsd[0] < 1e-4
    np.testing.assert_array_equal(T[:, 12], r.rmsd)
    ref_com = _check_records(traj, T, traj[0].cpu().numpy().astype(np.float64))
    # per-frame QCP rmsd of the sampled frames
    ref_c = O.centred_reference(traj[0].cpu().numpy().astype(np.float64))[1]
    for f in SAMPLE_FRAMES[1:4]:
        mob = traj[f].cpu().numpy().astype(np.float64)
        exp = O.CalcRMSDRotationalMatrix(ref_c, mob - mob.mean(axis=0), n_atoms, np.zeros(9), None)
        assert abs(r.rmsd[f] - exp) < 1e-9 * max(1.0, exp)
    atoms = _sampled_atoms(n_atoms)
    rows = traj[:, _t.as_tensor(atoms, device=traj.device)].cpu().numpy()
    mean, rmsf = _welford_rmsf(_aligned_rows(rows, T, ref_com))
    print(f"  C3 48 atoms: max|dmean| {np.abs(r.mean[atoms] - mean).max():.2e}, "
          f"max|dRMSF| {np.abs(r.rmsf[atoms] - rmsf).max():.2e} A")
    np.testing.assert_allclose(r.mean[atoms], mean, rtol=0, atol=TOL)
    np.testing.assert_allclose(r.rmsf[atoms], rmsf, rtol=0, atol=TOL)
    _release(traj)


def test_full_size_rmsf_py_two_sweeps():
    """RMSF.py's two sweeps (align="average") at 100k x 20k: sweep 1's
    records pinned on sampled frames and its average rebuilt on 48 atoms
    (RMSF.py:99-111); sweep 2's records pinned against the CPU QCP to the
    device average (RMSF.py:113-118), and the 48 atoms' RMSF rebuilt through
    RMSF.py:133-138 + 146, within 1e-6 A."""
    import torch as _t
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = N_FULL, NF_FULL
    traj = generate(Engine(), n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    r = RMSF(traj, align="average", collect_transforms=True).run().results
    T1, T2 = r.transforms_sweep1, r.transforms
    assert T1.shape == T2.shape == (nf, 16)
    atoms = _sampled_atoms(n_atoms)
    rows = traj[:, _t.as_tensor(atoms, device=traj.device)].cpu().numpy()
    # sweep 1: to frame 0; the average of the aligned frames
    ref_com1 = _check_records(traj, T1, traj[0].cpu().numpy().astype(np.float64), SAMPLE_FRAMES[::2])
    avg = _aligned_rows(rows, T1, ref_com1).astype(np.float64).sum(axis=0) / nf
    print(f"  sweep 1, 48 atoms: max|daverage| {np.abs(r.average[atoms] - avg).max():.2e} A")
    np.testing.assert_allclose(r.average[atoms], avg, rtol=0, atol=TOL)
    # sweep 2: to the device average
    ref_com2 = _check_records(traj, T2, np.asarray(r.average, dtype=np.float64), SAMPLE_FRAMES[1::2])
    mean, rmsf = _welford_rmsf(_aligned_rows(rows, T2, ref_com2))
    print(f"  sweep 2, 48 atoms: max|dmean| {np.abs(r.mean[atoms] - mean).max():.2e}, "
          f"max|dRMSF| {np.abs(r.rmsf[atoms] - rmsf).max():.2e} A")
    np.testing.assert_allclose(r.mean[atoms], mean, rtol=0, atol=TOL)
    np.testing.assert_allclose(r.rmsf[atoms], rmsf, rtol=0, atol=TOL)
    _release(traj)


def test_full_size_c3_strided_selection():
    """C3 at full size with a "CA-like" strided selection (every 10th atom,
    10k of 100k; SURVEY 8, "an optional strided fit subset"): the gathered
    superposition sums and the gathered aligned accumulate over 100k x 20k.
    Device R/COM of sampled frames against the CPU QCP on the whole
    selection (1e-9), then 48 selected atoms rebuilt through RMSF.py:133-138
    with the device's per-frame records (1e-6 A)."""
    import torch as _t
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = N_FULL, NF_FULL
    sel = np.arange(0, n_atoms, 10)
    traj = generate(Engine(), n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    r = RMSF(traj, select=sel, align="frame0", collect_transforms=True).run().results
    T = r.transforms
    assert T.shape == (nf, 16) and r.rmsf.shape == (len(sel),)
    sel_dev = _t.as_tensor(sel, device=traj.device)
    ref_full = traj[0][sel_dev].cpu().numpy().astype(np.float64)
    ref_com, ref_c = O.centred_reference(ref_full)
    for f in SAMPLE_FRAMES[::2]:
        mob = traj[f][sel_dev].cpu().numpy()
        com = O.center_of_mass(mob).astype(np.float64)
        R = O.get_rotation_matrix(ref_c, mob.astype(np.float64) - com, len(mob))
        np.testing.assert_allclose(T[f, 9:12], com, rtol=0, atol=1e-9, err_msg=f"COM of frame {f}")
        np.testing.assert_allclose(T[f, :9], R.reshape(-1), rtol=0, atol=1e-9, err_msg=f"R of frame {f}")
    pick = np.sort(np.random.default_rng(11).choice(len(sel), 48, replace=False))
    rows = traj[:, _t.as_tensor(sel[pick], device=traj.device)].cpu().numpy()
    mean, rmsf = _welford_rmsf(_aligned_rows(rows, T, ref_com))
    print(f"\n  C3 strided selection, 48 atoms: max|dmean| {np.abs(r.mean[pick] - mean).max():.2e}, "
          f"max|dRMSF| {np.abs(r.rmsf[pick] - rmsf).max():.2e} A")
    np.testing.assert_allclose(r.mean[pick], mean, rtol=0, atol=TOL)
    np.testing.assert_allclose(r.rmsf[pick], rmsf, rtol=0, atol=TOL)
    _release(traj)


def test_full_size_rmsf_py_selection_masses():
    """RMSF.py's two sweeps at full size over a strided selection with
    heterogeneous masses (RMSF.py:84,94,117,127's mass-weighted centres of
    mass; the QCP stays unweighted, as RMSF.py:48 passes weights=None).
    Sweep 1's records are pinned on sampled frames and its average rebuilt on
    48 atoms (RMSF.py:94-111); sweep 2's records are pinned against the CPU
    QCP to the device average (RMSF.py:113-118) and the 48 atoms' RMSF is
    rebuilt through RMSF.py:133-138 + 146 (1e-6 A)."""
    import torch as _t
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = N_FULL, NF_FULL
    sel = np.arange(3, n_atoms, 10)
    m = np.random.default_rng(5).uniform(1.0, 16.0, len(sel))
    traj = generate(Engine(), n_atoms, 0, nf, seed=0, motion=motion_table(1, nf))
    r = RMSF(traj, select=sel, masses=m, align="average", collect_transforms=True).run().results
    T1, T2 = r.transforms_sweep1, r.transforms
    sel_dev = _t.as_tensor(sel, device=traj.device)

    def check(T, ref_sel_f64, frames):
        ref_com, ref_c = O.centred_reference(ref_sel_f64, m)
        for f in frames:
            mob = traj[f][sel_dev].cpu().numpy()
            com = O.center_of_mass(mob, m).astype(np.float64)
            R = O.get_rotation_matrix(ref_c, mob.astype(np.float64) - com, len(mob))
            np.testing.assert_allclose(T[f, 9:12], com, rtol=0, atol=1e-9, err_msg=f"COM of frame {f}")
            np.testing.assert_allclose(T[f, :9], R.reshape(-1), rtol=0, atol=1e-9, err_msg=f"R of frame {f}")
        return ref_com

    ref_com1 = check(T1, traj[0][sel_dev].cpu().numpy().astype(np.float64), SAMPLE_FRAMES[::2])
    pick = np.sort(np.random.default_rng(12).choice(len(sel), 48, replace=False))
    rows = traj[:, _t.as_tensor(sel[pick], device=traj.device)].cpu().numpy()
    avg = _aligned_rows(rows, T1, ref_com1).astype(np.float64).sum(axis=0) / nf
    np.testing.assert_allclose(r.average[pick], avg, rtol=0, atol=TOL)
    ref_com2 = check(T2, np.asarray(r.average, dtype=np.float64), SAMPLE_FRAMES[1::2])
    mean, rmsf = _welford_rmsf(_aligned_rows(rows, T2, ref_com2))
    print(f"\n  RMSF.py sweeps, strided selection + masses, 48 atoms: max|daverage| "
          f"{np.abs(r.average[pick] - avg).max():.2e}, max|dRMSF| {np.abs(r.rmsf[pick] - rmsf).max():.2e} A")
    np.testing.assert_allclose(r.mean[pick], mean, rtol=0, atol=TOL)
    np.testing.assert_allclose(r.rmsf[pick], rmsf, rtol=0, atol=TOL)
    _release(traj)
