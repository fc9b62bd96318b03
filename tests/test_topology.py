"""CPU tier: the native GRO reader + selection fallback.
MDAnalysis is absent, so selections are checked against hand-built truth."""
import numpy as np
import pytest


@pytest.fixture
def gro(tmp_path):
    from rmsf_amd.topology import write_gro
    resids, resnames, names = [], [], []
    for r, rn in enumerate(["MET", "ARG", "ILE", "LYSH", "HISD"], start=1):
        for an in ["N", "H", "CA", "HA", "C", "O", "CB"]:
            resids.append(r), resnames.append(rn), names.append(an)
    for w in range(3):  # waters
        for an in ["OW", "HW1", "HW2"]:
            resids.append(6 + w), resnames.append("SOL"), names.append(an)
    resids.append(9), resnames.append("CA"), names.append("CA")  # a calcium ion
    n = len(names)
    rng = np.random.default_rng(0)
    frames = rng.uniform(0, 50, (3, n, 3)).astype(np.float32)
    path = str(tmp_path / "sys.gro")
    write_gro(path, resids, resnames, names, frames)
    return path, np.array(resids), np.array(resnames), np.array(names), frames


def test_read_gro(gro):
    from rmsf_amd.topology import GroTopology
    path, resids, resnames, names, frames = gro
    top = GroTopology(path)
    assert top.n_atoms == len(names) and top.frames.shape == frames.shape
    np.testing.assert_array_equal(top.resids, resids)
    assert list(top.names) == list(names) and list(top.resnames) == list(resnames)
    # MDAnalysis GROReader rounding: f32(text nm) then *10 in f32
    exp = (np.round(frames.astype(np.float64) / 10.0, 3).astype(np.float32) * np.float32(10.0))
    np.testing.assert_allclose(top.frames, exp, atol=1e-5)


def test_selections(gro):
    from rmsf_amd.topology import GroTopology
    path, resids, resnames, names, _ = gro
    top = GroTopology(path)
    ca = np.flatnonzero(names == "CA")
    prot = np.isin(resnames, ["MET", "ARG", "ILE", "LYSH", "HISD"])
    np.testing.assert_array_equal(top.select("protein and name CA"), np.flatnonzero(prot & (names == "CA")))
    assert len(top.select("name CA")) == len(ca)  # includes the calcium ion
    np.testing.assert_array_equal(top.select("not protein"), np.flatnonzero(~prot))
    np.testing.assert_array_equal(top.select("backbone"), np.flatnonzero(prot & np.isin(names, ["N", "CA", "C", "O"])))
    np.testing.assert_array_equal(top.select("resid 2-3 and name N C"),
                                  np.flatnonzero(np.isin(resids, [2, 3]) & np.isin(names, ["N", "C"])))
    np.testing.assert_array_equal(top.select("name H*"), np.flatnonzero(np.char.startswith(names.astype(str), "H")))
    np.testing.assert_array_equal(top.select("index 0:4 or bynum 10"), np.array([0, 1, 2, 3, 4, 9]))
    np.testing.assert_array_equal(top.select("(resname SOL or resname CA) and not name HW*"),
                                  np.flatnonzero(np.isin(resnames, ["SOL", "CA"]) & ~np.isin(names, ["HW1", "HW2"])))
    with pytest.raises(ValueError):
        top.select("around 5 protein")


def test_guess_masses_like_mdanalysis():
    """MDAnalysis' name -> element -> mass guess (upstream guessers; restated,
    unpinned): C-alphas are carbon (also a calcium ion *named* CA -- the
    upstream quirk), ion names go through the special-name table."""
    from rmsf_amd.topology import guess_atom_element, guess_masses
    cases = {"CA": "C", "N": "N", "OW": "O", "HW1": "H", "1HB": "H", "OC1": "O", "SD": "S", "CB": "C",
             "CLA": "CL", "SOD": "NA", "POT": "K", "CAL": "CA", "ZN": "ZN", "MW": "DUMMY", "NA+": "NA", "P": "P"}
    for name, el in cases.items():
        assert guess_atom_element(name) == el, name
    np.testing.assert_array_equal(guess_masses(["CA", "N", "O", "H", "S", "CAL", "XQ"]),
                                  [12.011, 14.007, 15.999, 1.008, 32.06, 40.08, 0.0])


def test_gro_topology_has_guessed_masses(gro):
    from rmsf_amd.topology import GroTopology, guess_masses
    path, _, _, names, _ = gro
    top = GroTopology(path)
    np.testing.assert_array_equal(top.masses, guess_masses(names))
    assert top.masses[list(names).index("CA")] == 12.011
