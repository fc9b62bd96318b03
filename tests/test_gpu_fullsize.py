"""GPU tier at BASELINE.json's full sizes, checked through size-independent
properties: sampled atoms regenerated bit-exactly on the CPU (counter-based
generator) against an independent two-pass variance, the analytic
sqrt(3)*sigma of the generator, invariance under the frame-tile split, and
per-frame QCP rmsd of sampled frames against the CPU restatement.

  C2  100k atoms x 20k frames, no alignment           (24 GB in HBM)
  C3  100k atoms x 20k frames, QCP to frame 0         (24 GB)
  C4  1M atoms x 2.5k frames (one GPU's share at N=8) (30 GB)
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
    _release(traj)


def test_full_size_aligned_c3():
    from rmsf_amd import RMSF
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table
    n_atoms, nf = 100_000, 20_000
    mt = motion_table(1, nf)
    traj = generate(Engine(), n_atoms, 0, nf, seed=0, motion=mt)
    r = RMSF(traj, align="frame0", collect_rmsd=True).run().results
    assert r.rmsd.shape == (nf,) and r.rmsd[0] < 1e-4
    # rigid motions removed: what is left is the generator's noise
    np.testing.assert_allclose(r.rmsf, SY.expected_rmsf(0, np.arange(n_atoms)), rtol=0.05)
    # per-frame QCP rmsd of sampled frames against the CPU restatement
    ref = traj[0].cpu().numpy().astype(np.float64)
    ref_c = ref - ref.mean(axis=0)
    for f in (1, 777, 12345, nf - 1):
        mob = traj[f].cpu().numpy().astype(np.float64)
        mob_c = mob - mob.mean(axis=0)
        rot = np.zeros(9)
        exp = O.CalcRMSDRotationalMatrix(ref_c, mob_c, n_atoms, rot, None)
        assert abs(r.rmsd[f] - exp) < 1e-9 * max(1.0, exp)
    _release(traj)
