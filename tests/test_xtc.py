"""CPU tier: the native XTC codec (csrc/xtc.cpp, host-only C++).

No reference XTC file exists here (MDAnalysisTests is not installed), so the
format is UNPINNED; these tests pin the codec against (a) the exact
quantisation arithmetic of a write -> read round trip, computed in numpy, and
(b) an independent pure-Python decoder (oracle/xtc_py.py)."""
import os

import numpy as np
import pytest

from oracle import xtc_py


def _protein_like(rng, n_atoms, n_frames, scale=1.0):
    """Chains of ~1.5 A bonds plus 3-atom water clusters (exercises the
    run-length/small-difference and water-swap paths), drifting per frame."""
    base = np.cumsum(rng.normal(0, 1.5, (n_atoms, 3)), axis=0) * scale + 40.0
    w = n_atoms // 3
    base[-3 * (w // 2):] = np.repeat(rng.uniform(0, 80, (w // 2, 3)), 3, axis=0) + rng.normal(0, 0.9, (3 * (w // 2), 3))
    return np.stack([base + rng.normal(0, 0.3, base.shape) for _ in range(n_frames)]).astype(np.float32)


@pytest.fixture
def tmpfile(tmp_path):
    return str(tmp_path / "t.xtc")


@pytest.mark.parametrize("n_atoms,prec", [(10, 1000.0), (500, 1000.0), (3341, 1000.0), (1000, 100.0), (2000, 10000.0)])
def test_round_trip_exact_quantisation(tmpfile, n_atoms, prec):
    from rmsf_amd.xtc import XTCFile, write_xtc
    rng = np.random.default_rng(n_atoms)
    x = _protein_like(rng, n_atoms, 7)
    write_xtc(tmpfile, x, precision=prec)
    with XTCFile(tmpfile) as f:
        assert (f.n_atoms, f.n_frames) == (n_atoms, 7)
        got = f.read(n_threads=3)
    np.testing.assert_array_equal(got, xtc_py.quantize_expected(x, prec))
    # half a quantum (10/prec A) plus f32 rounding of the A<->nm conversions
    assert np.abs(got - x).max() <= 5.0 / prec + 2e-5


def test_native_matches_python_decoder(tmpfile):
    from rmsf_amd.xtc import XTCFile, write_xtc
    rng = np.random.default_rng(7)
    x = _protein_like(rng, 777, 5)
    write_xtc(tmpfile, x)
    with XTCFile(tmpfile) as f:
        native = f.read()
    np.testing.assert_array_equal(native, xtc_py.read_xtc(tmpfile))


def test_small_systems_uncompressed(tmpfile):
    """<= 9 atoms are stored as raw floats (no quantisation)."""
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = np.random.default_rng(1).uniform(-50, 50, (4, 9, 3)).astype(np.float32)
    write_xtc(tmpfile, x)
    with XTCFile(tmpfile) as f:
        got = f.read()
    np.testing.assert_array_equal(got, xtc_py.quantize_expected(x))
    np.testing.assert_array_equal(got, xtc_py.read_xtc(tmpfile))


@pytest.mark.parametrize("kind", ["two_clusters", "no_close_pairs"])
def test_large_range_path(tmpfile, kind):
    """Coordinate ranges above 0xffffff quanta switch to per-axis bit sizes;
    "no_close_pairs" drives the magicints index to the end of the table."""
    from rmsf_amd.xtc import XTCFile, write_xtc
    rng = np.random.default_rng(3)
    if kind == "two_clusters":  # two chains 80,000 nm apart
        x = _protein_like(rng, 400, 2)
        x[:, 200:] += np.float32(8e5)
        x[:, :200] -= np.float32(8e4)
    else:
        x = rng.uniform(-4e5, 4e5, (2, 300, 3)).astype(np.float32)
    write_xtc(tmpfile, x, precision=1000.0)
    with XTCFile(tmpfile) as f:
        got = f.read()
    np.testing.assert_array_equal(got, xtc_py.quantize_expected(x))
    np.testing.assert_array_equal(got, xtc_py.read_xtc(tmpfile))


def test_selection_step_and_frame_info(tmpfile):
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = _protein_like(np.random.default_rng(5), 400, 11)
    write_xtc(tmpfile, x, box=np.diag([60.0, 70.0, 80.0]))
    sel = np.array([3, 0, 399, 17])
    with XTCFile(tmpfile) as f:
        full = f.read()
        part = f.read(start=2, n=3, step=3, sel=sel)
        step, time, box = f.frame_info(5)
    np.testing.assert_array_equal(part, full[2:12:3][:, sel])
    assert step == 5 and time == 5.0
    np.testing.assert_allclose(np.diag(box), [6.0, 7.0, 8.0], rtol=1e-6)  # stored in nm


def test_append_and_truncated_tail(tmpfile):
    from rmsf_amd.xtc import XTCFile, write_xtc
    x = _protein_like(np.random.default_rng(6), 300, 3)
    write_xtc(tmpfile, x[:2])
    write_xtc(tmpfile, x[2:], append=True)
    size = os.path.getsize(tmpfile)
    with open(tmpfile, "ab") as fh:
        fh.write(open(tmpfile, "rb").read()[: size // 5])  # a partial 4th frame
    with XTCFile(tmpfile) as f:
        assert f.n_frames == 3  # the truncated tail frame is ignored
        np.testing.assert_array_equal(f.read(), xtc_py.quantize_expected(x))


def test_rejects_non_xtc(tmp_path):
    from rmsf_amd import RmsfError
    from rmsf_amd.xtc import XTCFile
    p = tmp_path / "x.xtc"
    p.write_bytes(b"\x00" * 200)
    with pytest.raises(RmsfError, match="not an XTC"):
        XTCFile(str(p))
