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


@pytest.mark.parametrize("select", ["protein and name CA", "backbone"])
def test_script_mode_gro_xtc_native(tmp_path, select):
    """RMSF.py's own input pair (GRO topology + XTC trajectory, "protein and
    name CA", two-sweep average alignment) end to end without MDAnalysis; the
    centre of mass weights with masses guessed from the GRO names, as
    MDAnalysis does (a mixed-element backbone selection exercises it)."""
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
                        "--trajectory", xtc, "--out", out, "--select", select], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Process:  0 --> Frames:" in r.stdout
    top = GroTopology(gro)
    sel = top.select(select)
    assert len(sel) == (n_res if select.endswith("CA") else 4 * n_res)
    assert len(set(top.masses[sel])) == (1 if select.endswith("CA") else 3)
    with XTCFile(xtc) as f:
        dec = f.read()
    exp = O.rmsf_script(dec, sel, top.masses[sel], size=1, align="average")["rmsf"]
    np.testing.assert_allclose(np.load(out), exp, rtol=0, atol=1e-6)


def test_script_mode_psf_dcd_native(tmp_path):
    """BASELINE config C1's file pair: the adk shape (3341 atoms, 214 CA, 98
    frames) as PSF + DCD, RMSF.py's defaults (protein and name CA, mass-
    weighted COM from the PSF masses, two-sweep average), without MDAnalysis;
    and RMSF() reading the .dcd directly, with a frame slice."""
    import subprocess
    import sys

    from conftest import ROOT
    from oracle import synth as SY
    from rmsf_amd import RMSF
    from rmsf_amd.dcd import write_dcd
    from rmsf_amd.synth import motion_table
    from rmsf_amd.topology import PsfTopology, write_psf
    n_res, n_atoms, nf = 214, 3341, 98
    per = (n_atoms - 400) // n_res  # protein atoms per residue; the rest is solvent
    resids = np.concatenate([np.repeat(np.arange(1, n_res + 1), per),
                             np.arange(n_res + 1, n_res + 1 + n_atoms - per * n_res)])
    resnames = np.concatenate([np.array(["MET", "ARG", "ILE", "HSD", "GLY"])[np.repeat(np.arange(n_res), per) % 5],
                               ["TIP3"] * (n_atoms - per * n_res)])
    base = ["N", "CA", "C", "O", "CB", "CG", "CD", "NE", "CZ", "NH1", "NH2", "HA", "HB1"]
    names = np.concatenate([np.tile(base[:per], n_res), ["OH2"] * (n_atoms - per * n_res)])
    masses = np.array([{"N": 14.007, "O": 15.999, "OH2": 15.999}.get(a, 12.011) for a in names])
    x = SY.frames(31, n_atoms, 0, nf, motion_table(32, nf))
    psf, dcd, out = str(tmp_path / "adk.psf"), str(tmp_path / "adk.dcd"), str(tmp_path / "rmsf.npy")
    write_psf(psf, resids, resnames, names, masses)
    write_dcd(dcd, x, box=(60.0, 90.0, 60.0, 90.0, 90.0, 60.0))
    r = subprocess.run([sys.executable, f"{ROOT}/mdanalysis-mpi_amd/rmsf_mi355x.py", "--topology", psf,
                        "--trajectory", dcd, "--out", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    top = PsfTopology(psf)
    sel = top.select("protein and name CA")
    assert len(sel) == n_res
    exp = O.rmsf_script(x, sel, top.masses[sel], size=1, align="average")["rmsf"]
    np.testing.assert_allclose(np.load(out), exp, rtol=0, atol=1e-6)
    got = RMSF(dcd, select=sel, masses=top.masses[sel], align="frame0").run(start=3, stop=90, step=2)
    exp = O.rmsf_script(x, sel, top.masses[sel], size=1, align="frame0", start=3, stop=90, step=2)["rmsf"]
    np.testing.assert_allclose(got.results.rmsf, exp, rtol=0, atol=1e-6)


@pytest.mark.parametrize("cache", [False, True])
def test_dcd_streamed_equals_host_array(tmp_path, cache):
    """DcdSource reads each batch's selected rows from the memory-mapped file
    (RMSF.py:92,124's reader) instead of the whole file up front: same frames,
    same bits as the host array of the same trajectory."""
    from oracle import synth as SY
    from rmsf_amd import RMSF
    from rmsf_amd.dcd import write_dcd
    from rmsf_amd.sources import DcdSource, HostSource
    from rmsf_amd.synth import motion_table

    x = SY.frames(5, 700, 0, 61, motion_table(6, 61))
    sel = np.arange(3, 700, 5)
    p = str(tmp_path / "t.dcd")
    write_dcd(p, x)
    kw = dict(start=2, stop=59, step=3)
    src = DcdSource(p, sel, batch_frames=4, cache=cache)
    got = RMSF(src, align="average").run(**kw).results
    ref = RMSF(HostSource(x, sel, batch_frames=4), align="average").run(**kw).results
    np.testing.assert_array_equal(got.rmsf, ref.rmsf)
    np.testing.assert_array_equal(got.average, ref.average)
    assert (src.cache is not None) == cache
