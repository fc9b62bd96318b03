"""GPU tier: RMSF straight from an XTC file (native frame-parallel decode into
the pinned stager, DMA, kernels) equals RMSF of the decoded frames, and the
oracle restatement of RMSF.py on them."""
import numpy as np
import pytest
import torch

from oracle import rmsf_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("align", [None, "frame0", "average"])
def test_rmsf_from_xtc(tmp_path, align):
    from oracle import synth as SY
    from rmsf_amd import RMSF
    from rmsf_amd.synth import motion_table
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = SY.frames(12, 2000, 0, 37, motion_table(13, 37))
    path = str(tmp_path / "traj.xtc")
    write_xtc(path, x)
    sel = np.arange(1, 2000, 7)
    with XTCFile(path) as f:
        dec = f.read()
    got = RMSF(path, select=sel, align=align, batch_frames=5).run()
    ref = RMSF(torch.tensor(dec, device="cuda"), select=sel, align=align).run()
    np.testing.assert_array_equal(got.results.n_frames, 37)
    np.testing.assert_allclose(got.results.rmsf, ref.results.rmsf, rtol=0, atol=1e-9)
    exp = O.rmsf_script(dec, sel, None, size=1, align=align)["rmsf"]
    np.testing.assert_allclose(got.results.rmsf, exp, rtol=0, atol=1e-6)
    s = RMSF(path, select=sel, align=align).run(start=2, stop=30, step=3)
    exp = O.rmsf_script(dec, sel, None, size=1, align=align, start=2, stop=30, step=3)["rmsf"]
    np.testing.assert_allclose(s.results.rmsf, exp, rtol=0, atol=1e-6)


def test_script_mode_gro_xtc_native(tmp_path):
    """RMSF.py's own input pair (GRO topology + XTC trajectory, "protein and
    name CA", two-sweep average alignment) end to end without MDAnalysis."""
    import subprocess
    import sys

    from conftest import ROOT
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table
    from rmsf_amd.topology import GroTopology, write_gro
    from rmsf_amd.xtc import XTCFile, write_xtc
    n_res = 60
    resids = np.repeat(np.arange(1, n_res + 1), 5)
    resnames = np.array(["ALA", "GLY", "LYSH", "HISD", "MET"] * 12)[np.repeat(np.arange(n_res), 5) % 60]
    names = np.tile(["N", "CA", "C", "O", "CB"], n_res)
    extra = 50  # solvent + a calcium ion named CA
    resids = np.concatenate([resids, np.arange(n_res + 1, n_res + 1 + extra)])
    resnames = np.concatenate([resnames, ["SOL"] * (extra - 1) + ["CA"]])
    names = np.concatenate([names, ["OW"] * (extra - 1) + ["CA"]])
    n = len(names)
    x = SY.frames(21, n, 0, 25, motion_table(22, 25))
    gro, xtc, out = str(tmp_path / "s.gro"), str(tmp_path / "s.xtc"), str(tmp_path / "rmsf.npy")
    write_gro(gro, resids, resnames, names, x[0])
    write_xtc(xtc, x)
    r = subprocess.run([sys.executable, f"{ROOT}/mdanalysis-mpi_amd/rmsf_mi355x.py", "--topology", gro,
                        "--trajectory", xtc, "--out", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Process:  0 --> Frames:" in r.stdout
    sel = GroTopology(gro).select("protein and name CA")
    assert len(sel) == n_res
    with XTCFile(xtc) as f:
        dec = f.read()
    exp = O.rmsf_script(dec, sel, None, size=1, align="average")["rmsf"]
    np.testing.assert_allclose(np.load(out), exp, rtol=0, atol=1e-6)
