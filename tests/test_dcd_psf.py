"""PSF topology + DCD trajectory (BASELINE config C1's adk PSF/DCD pair).

CPU tier.  No DCD/PSF file of the reference exists here (MDAnalysisTests is
not installed), so the formats are unpinned: the reader is checked against
its writer (round trips with and without unit cells, both byte orders, fixed
atoms) and against an independent record-by-record parse written here with
``struct``; the PSF parser against the MDAnalysis selection semantics it
feeds (``protein and name CA``, masses)."""
import struct

import numpy as np
import pytest

from rmsf_amd.dcd import DCDFile, write_dcd
from rmsf_amd.topology import PsfTopology, write_psf


def _independent_dcd(path):
    """Plain struct walk over the records: (n_atoms, frames [n, n_atoms, 3])."""
    b = open(path, "rb").read()
    e = "<" if struct.unpack("<i", b[:4])[0] == 84 else ">"
    icntrl = struct.unpack(e + "20i", b[8:88])
    charmm, cell, namnf = icntrl[19] != 0, icntrl[19] != 0 and icntrl[10] != 0, icntrl[8]
    p = 92
    tlen = struct.unpack(e + "i", b[p:p + 4])[0]
    p += 8 + tlen
    natoms = struct.unpack(e + "i", b[p + 4:p + 8])[0]
    p += 12
    free = None
    if namnf:
        nfree = natoms - namnf
        free = np.array(struct.unpack(e + f"{nfree}i", b[p + 4:p + 4 + 4 * nfree])) - 1
        p += 8 + 4 * nfree
    frames = []
    while p < len(b):
        if cell:
            p += 56
        n = natoms if (not frames or free is None) else len(free)
        xyz = np.zeros((natoms, 3), np.float32) if not frames else frames[0].copy()
        for c in range(3):
            ln = struct.unpack(e + "i", b[p:p + 4])[0]
            assert ln == 4 * n
            v = np.array(struct.unpack(e + f"{n}f", b[p + 4:p + 4 + 4 * n]), np.float32)
            if n == natoms:
                xyz[:, c] = v
            else:
                xyz[free, c] = v
            p += 8 + 4 * n
        frames.append(xyz)
    return natoms, np.stack(frames)


@pytest.mark.parametrize("box", [None, (60.0, 90.0, 60.0, 90.0, 90.0, 60.0)])
@pytest.mark.parametrize("order", ["<", ">"])
def test_dcd_round_trip(tmp_path, box, order):
    rng = np.random.default_rng(3)
    x = rng.uniform(-50, 50, (7, 333, 3)).astype(np.float32)
    p = str(tmp_path / "t.dcd")
    write_dcd(p, x, box=box, byteorder=order)
    with DCDFile(p) as f:
        assert (f.n_atoms, f.n_frames, f.has_cell) == (333, 7, box is not None)
        np.testing.assert_array_equal(f.read(), x)
        np.testing.assert_array_equal(f.read(2, 3, 2), x[2:8:2][:3])
        sel = np.array([3, 5, 200])
        np.testing.assert_array_equal(f.read(sel=sel), x[:, sel])
    na, ind = _independent_dcd(p)
    assert na == 333
    np.testing.assert_array_equal(ind, x)


def test_dcd_xplor_and_fixed_atoms(tmp_path):
    rng = np.random.default_rng(4)
    x = rng.uniform(-50, 50, (5, 40, 3)).astype(np.float32)
    fixed = np.array([0, 7, 8, 39])
    x[1:, fixed] = x[0, fixed]  # fixed atoms keep frame 0's coordinates
    p = str(tmp_path / "f.dcd")
    write_dcd(p, x, fixed=fixed, charmm=False)
    with DCDFile(p) as f:
        assert not f.charmm and f.n_frames == 5
        np.testing.assert_array_equal(f.read(), x)
        np.testing.assert_array_equal(f.read(3, 1), x[3:4])
    np.testing.assert_array_equal(_independent_dcd(p)[1], x)


def test_dcd_rejects_garbage(tmp_path):
    p = str(tmp_path / "g.dcd")
    open(p, "wb").write(b"\x00" * 200)
    with pytest.raises(ValueError):
        DCDFile(p)
    x = np.zeros((2, 10, 3), np.float32)
    write_dcd(p, x)
    b = bytearray(open(p, "rb").read())
    b[-4:] = b"\x01\x02\x03\x04"  # break the last record's closing marker... and its length check on read
    b[-4 - 40 - 4:-4 - 40] = struct.pack("<i", 12)  # Z record of frame 1 claims 3 atoms
    open(p, "wb").write(bytes(b))
    with pytest.raises(ValueError):
        DCDFile(p).read()


@pytest.mark.parametrize("box", [None, (60.0, 90.0, 60.0, 90.0, 90.0, 60.0)])
def test_dcd_plane_ptrs(tmp_path, box):
    """The addresses DcdSource hands to rmsf_stager_stage_planes: frame f's X
    record, Y and Z records plane_stride floats further on -- read back
    through them, they give read()'s frames; markers are checked; files the
    plane path cannot read in place (other byte order, fixed atoms) return
    None and keep the read() path."""
    import ctypes

    rng = np.random.default_rng(5)
    x = rng.uniform(-50, 50, (6, 101, 3)).astype(np.float32)
    p = str(tmp_path / "p.dcd")
    write_dcd(p, x, box=box)
    with DCDFile(p) as f:
        frames = np.array([0, 2, 5, 3])
        ptrs, ps = f.plane_ptrs(frames)
        assert ps == 101 + 2 and ptrs.dtype == np.uint64
        for k, fr in enumerate(frames):
            buf = (ctypes.c_float * (2 * ps + 101)).from_address(int(ptrs[k]))
            planes = np.frombuffer(buf, dtype=np.float32)
            got = np.stack([planes[c * ps:c * ps + 101] for c in range(3)], axis=1)
            np.testing.assert_array_equal(got, x[fr])
        with pytest.raises(IndexError):
            f.plane_ptrs([6])
    b = bytearray(open(p, "rb").read())
    with DCDFile(p) as f:
        pos = f._data0 + 2 * f._full + (56 if box else 0) + (8 + 4 * 101)  # frame 2's Y record marker
    b[pos:pos + 4] = struct.pack("<i", 8)
    q = str(tmp_path / "bad.dcd")
    open(q, "wb").write(bytes(b))
    with DCDFile(q) as f:
        f.plane_ptrs([0, 1])
        with pytest.raises(ValueError, match="markers"):
            f.plane_ptrs([1, 2])
    write_dcd(p, x, byteorder=">")
    with DCDFile(p) as f:
        assert f.plane_ptrs([0]) is None
    fixed = np.array([1, 4])
    x[1:, fixed] = x[0, fixed]
    write_dcd(p, x, fixed=fixed)
    with DCDFile(p) as f:
        assert f.plane_ptrs([0]) is None


def test_psf_topology_selection(tmp_path):
    resids = [1, 1, 1, 2, 2, 2, 3, 4, 4]
    resnames = ["MET", "MET", "MET", "HSD", "HSD", "HSD", "TIP3", "POPC", "POPC"]
    names = ["N", "CA", "C", "N", "CA", "C", "OH2", "P", "C21"]
    masses = [14.007, 12.011, 12.011, 14.007, 12.011, 12.011, 15.999, 30.974, 12.011]
    p = str(tmp_path / "t.psf")
    write_psf(p, resids, resnames, names, masses)
    t = PsfTopology(p)
    assert t.n_atoms == 9
    np.testing.assert_array_equal(t.select("protein and name CA"), [1, 4])
    np.testing.assert_array_equal(t.select("backbone"), [0, 1, 2, 3, 4, 5])
    np.testing.assert_array_equal(t.select("resname POPC and not name P"), [8])
    np.testing.assert_array_equal(t.masses[t.select("name CA")], [12.011, 12.011])
    bad = str(tmp_path / "bad.psf")
    open(bad, "w").write("not a psf\n")
    with pytest.raises(ValueError):
        PsfTopology(bad)
