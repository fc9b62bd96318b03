"""Minimal GRO / PSF topologies + selection fallback.

RMSF.py builds ``mda.Universe(GRO, XTC)`` (RMSF.py:34,56) and selects
``"protein and name CA"`` (RMSF.py:77,116,120,126); BASELINE config C1 names
the PSF/DCD pair of the same adk system.  When MDAnalysis is not installed,
this module reads the GRO or PSF file itself and evaluates a subset of the
MDAnalysis selection language, so the whole script runs natively:

    top = GroTopology("adk.gro")                   # or PsfTopology("adk.psf")
    sel = top.select("protein and name CA")        # sorted atom indices
    RMSF("adk.xtc", select=sel, align="average").run()   # or "adk.dcd"

Supported selection grammar (MDAnalysis keywords and precedence: ``not`` >
``and`` > ``or``, parentheses): ``all``, ``none``, ``protein``, ``backbone``
(protein and name N CA C O), ``name``/``resname`` with shell-style wildcards,
``resid a``/``resid a-b``/``resid a:b``, ``index``/``bynum`` (0- / 1-based,
ranges).  ``protein`` uses MDAnalysis' ProteinSelection residue-name set as
far as restated here (standard, CHARMM, GROMACS OPLS/GROMOS/AMBER variants).
Host-only pure Python; results are plain index arrays, so selections made by
MDAnalysis (``ag.indices``) can always be passed instead.  Parity with
MDAnalysis selections is UNPINNED here (MDAnalysis absent).
"""
from __future__ import annotations

import fnmatch
import re

import numpy as np

# MDAnalysis ProteinSelection.prot_res (restated; upstream not vendored)
PROTEIN_RESNAMES = frozenset("""
ALA ARG ASN ASP CYS GLN GLU GLY HSD HSE HSP ILE LEU LYS MET PHE PRO SER THR TRP TYR VAL ALAD
HIS MSE
ARGN ASPH CYS2 CYSH QLN PGLU GLUH HIS1 HISD HISE HISH LYSH
ASN1 CYS1 HISA HISB HIS2
HID HIE HIP ORN DAB LYN HYP CYM CYX ASH GLH ACE NME
NALA NGLY NSER NTHR NLEU NILE NVAL NASN NGLN NARG NHID NHIE NHIP NTRP NPHE NTYR NGLU NASP NLYS NPRO NCYS NCYX NMET
CALA CGLY CSER CTHR CLEU CILE CVAL CASN CGLN CARG CHID CHIE CHIP CTRP CPHE CTYR CGLU CASP CLYS CPRO CCYS CCYX CMET
CME ASF
""".split())
BACKBONE_NAMES = frozenset(["N", "CA", "C", "O"])

# MDAnalysis' mass guessing (upstream topology/guessers.py + tables.py;
# restated, not vendored -- parity UNPINNED here, MDAnalysis absent).  A GRO
# file carries no masses, so MDAnalysis guesses each atom's element from its
# name and takes the element's mass; RMSF.py's center_of_mass (RMSF.py:84,
# 94,117,127) weights with those.
#   tables.atomelements: special atom names -> element
_ATOM_ELEMENTS = {
    "BR": "BR", "CAL": "CA", "C0": "CA", "CA2+": "CA", "CES": "CS", "CLA": "CL", "CLAL": "CL", "CL": "CL",
    "CL-": "CL", "IOD": "I", "FE": "FE", "FE2": "FE", "LIT": "LI", "LI": "LI", "LI+": "LI", "QL": "LI",
    "MG": "MG", "MG2+": "MG", "K": "K", "POT": "K", "K+": "K", "QK": "K", "SOD": "NA", "NA": "NA",
    "NA+": "NA", "QN": "NA", "ZN": "ZN", "CU": "CU", "CS": "CS", "CS+": "CS", "QC": "CE", "RB": "RB",
    "QR": "RB", "BC": "C", "AC": "C", "MW": "DUMMY",
}
#   tables.elements: the elements a name may be cut down to
_ELEMENTS = frozenset(["H", "LI", "BE", "B", "C", "N", "O", "F", "NA", "MG", "AL", "P", "SI", "S", "CL", "K"])
#   tables.masses (the elements above and the ion names' elements)
ELEMENT_MASSES = {
    "H": 1.008, "LI": 6.941, "BE": 9.012182, "B": 10.811, "C": 12.011, "N": 14.007, "O": 15.999,
    "F": 18.9984032, "NA": 22.989768, "MG": 24.305, "AL": 26.981539, "SI": 28.0855, "P": 30.973762,
    "S": 32.06, "CL": 35.45, "K": 39.10, "CA": 40.08, "FE": 55.847, "CU": 63.546, "ZN": 65.39, "BR": 79.904,
    "RB": 85.4678, "I": 126.90447, "CS": 132.90, "CE": 140.115, "DUMMY": 0.0,
}


def guess_atom_element(name: str) -> str:
    """MDAnalysis ``guess_atom_element``: the special-name table first, then
    the name without charge symbols and digits cut down to a known element
    (whole, without its last or first letter, else from the right)."""
    if name == "":
        return ""
    up = name.upper()
    if up in _ATOM_ELEMENTS:
        return _ATOM_ELEMENTS[up]
    no_symbols = re.sub(r"[*+-]", "", name)
    nm = re.sub(r"[0-9]", "", no_symbols).upper()
    if nm in _ATOM_ELEMENTS:
        return _ATOM_ELEMENTS[nm]
    while nm:
        if nm in _ELEMENTS:
            return nm
        if nm[:-1] in _ELEMENTS:
            return nm[:-1]
        if nm[1:] in _ELEMENTS:
            return nm[1:]
        if len(nm) <= 2:
            return nm[0]
        nm = nm[:-1]
    return no_symbols


def guess_masses(names) -> np.ndarray:
    """f64 masses from atom names (MDAnalysis ``guess_masses(guess_types(names))``;
    unknown elements get 0.0, as upstream)."""
    return np.array([ELEMENT_MASSES.get(guess_atom_element(str(n)).upper(), 0.0) for n in names], dtype=np.float64)


class Topology:
    """Per-atom resids, resnames, names (and masses when the file has them)."""

    resids: np.ndarray
    resnames: np.ndarray
    names: np.ndarray
    masses: np.ndarray | None = None
    n_atoms: int

    def select(self, selection: str) -> np.ndarray:
        """Sorted unique atom indices (MDAnalysis ordering) matching ``selection``."""
        mask = _Parser(selection, self).parse()
        return np.flatnonzero(mask)


class PsfTopology(Topology):
    """The atoms of a CHARMM/NAMD/X-PLOR .psf file (the ``!NATOM`` section:
    id, segid, resid, resname, name, type, charge, mass, ...), as MDAnalysis'
    PSFParser reads them: standard and EXT layouts are both whitespace
    separated; resids keep their leading integer (insertion codes dropped);
    masses are float64 (MDAnalysis keeps them as read)."""

    def __init__(self, path: str):
        self.path = path
        lines = open(path).read().splitlines()
        if not lines or not lines[0].startswith("PSF"):
            raise ValueError(f"{path}: not a PSF file (first line must start with 'PSF')")
        for k, line in enumerate(lines):
            if "!NATOM" in line:
                n = int(line.split()[0])
                body = lines[k + 1:k + 1 + n]
                break
        else:
            raise ValueError(f"{path}: no !NATOM section")
        if len(body) < n:
            raise ValueError(f"{path}: !NATOM announces {n} atoms, {len(body)} lines follow")
        resids, resnames, names, masses = [], [], [], []
        for line in body:
            f = line.split()
            if len(f) < 8:
                raise ValueError(f"{path}: short atom line {line!r}")
            m = re.match(r"-?\d+", f[2])
            resids.append(int(m.group(0)) if m else 0)
            resnames.append(f[3])
            names.append(f[4])
            masses.append(float(f[7]))
        self.resids = np.array(resids, dtype=np.int64)
        self.resnames = np.array(resnames, dtype=object)
        self.names = np.array(names, dtype=object)
        self.masses = np.array(masses, dtype=np.float64)
        self.n_atoms = n


def write_psf(path: str, resids, resnames, names, masses=None, segid="PROT", title="rmsf_amd"):
    """Write a minimal standard-layout .psf (atoms only; tests/tools)."""
    masses = np.full(len(names), 12.011) if masses is None else np.asarray(masses, dtype=np.float64)
    with open(path, "w") as fh:
        fh.write(f"PSF\n\n{1:8d} !NTITLE\n* {title}\n\n{len(names):8d} !NATOM\n")
        for k, (ri, rn, an, m) in enumerate(zip(resids, resnames, names, masses)):
            fh.write(f"{k + 1:8d} {segid:<4s} {int(ri):<4d} {rn:<4s} {an:<4s} {an[:4]:<4s} {0.0:10.6f} "
                     f"{m:13.4f} {0:11d}\n")
        fh.write(f"\n{0:8d} !NBOND: bonds\n\n")


class GroTopology(Topology):
    """Atoms (resid, resname, name) and the frames of a .gro file.

    ``positions`` follow MDAnalysis' GROReader rounding: the text is parsed
    into float32 nm, then converted in place to Angstrom (x10 in float32).
    ``masses`` are guessed from the atom names as MDAnalysis' GROParser does
    (``guess_masses``), so a mass-weighted centre of mass matches RMSF.py's
    for any selection, not only uniform-mass ones."""

    def __init__(self, path: str):
        self.path = path
        frames, atoms = self._parse(path)
        self.resids = np.array([a[0] for a in atoms], dtype=np.int64)
        self.resnames = np.array([a[1] for a in atoms], dtype=object)
        self.names = np.array([a[2] for a in atoms], dtype=object)
        self.masses = guess_masses(self.names)
        self.n_atoms = len(atoms)
        self.frames = np.stack(frames)  # [n_frames, n_atoms, 3] float32 Angstrom

    @property
    def positions(self) -> np.ndarray:
        return self.frames[0]

    @staticmethod
    def _parse(path):
        lines = open(path).read().splitlines()
        frames, atoms = [], None
        i = 0
        while i + 1 < len(lines):
            n = int(lines[i + 1].split()[0])
            body = lines[i + 2:i + 2 + n]
            if len(body) < n:
                break
            # coordinate field width from the decimal-point spacing (GRO variable precision)
            first = body[0]
            d0 = first.find(".", 20)
            d1 = first.find(".", d0 + 1)
            cs = d1 - d0 if d0 > 0 and d1 > 0 else 8
            xyz = np.empty((n, 3), dtype=np.float32)
            rows = []
            for k, line in enumerate(body):
                if atoms is None:
                    rows.append((int(line[0:5]), line[5:10].strip(), line[10:15].strip()))
                for c in range(3):
                    xyz[k, c] = float(line[20 + cs * c:20 + cs * (c + 1)])
            if atoms is None:
                atoms = rows
            elif n != len(atoms):
                raise ValueError(f"{path}: frame {len(frames)} has {n} atoms, expected {len(atoms)}")
            xyz *= np.float32(10.0)  # nm -> Angstrom, in place in float32 (MDAnalysis convert_pos_from_native)
            frames.append(xyz)
            i += 2 + n + 1  # title, count, atoms, box
        if not frames:
            raise ValueError(f"{path}: no complete GRO frame")
        return frames, atoms


# ---------------------------------------------------------------------------
_TOKEN = re.compile(r"\(|\)|[^\s()]+")


class _Parser:
    """Recursive-descent evaluation: or_expr := and_expr ('or' and_expr)*,
    and_expr := unary ('and' unary)*, unary := 'not' unary | atom."""

    KEYWORDS = {"and", "or", "not", "(", ")"}
    SELECTORS = {"all", "none", "protein", "backbone", "name", "resname", "resid", "index", "bynum"}

    def __init__(self, text: str, top: Topology):
        self.tok = _TOKEN.findall(text)
        self.i = 0
        self.top = top

    def peek(self):
        return self.tok[self.i] if self.i < len(self.tok) else None

    def take(self):
        t = self.peek()
        if t is None:
            raise ValueError("unexpected end of selection")
        self.i += 1
        return t

    def parse(self) -> np.ndarray:
        m = self.or_expr()
        if self.peek() is not None:
            raise ValueError(f"unexpected token {self.peek()!r} in selection")
        return m

    def or_expr(self):
        m = self.and_expr()
        while self.peek() == "or":
            self.take()
            m = m | self.and_expr()
        return m

    def and_expr(self):
        m = self.unary()
        while self.peek() == "and":
            self.take()
            m = m & self.unary()
        return m

    def unary(self):
        if self.peek() == "not":
            self.take()
            return ~self.unary()
        if self.peek() == "(":
            self.take()
            m = self.or_expr()
            if self.take() != ")":
                raise ValueError("missing ')' in selection")
            return m
        return self.atom()

    def _values(self):
        vals = []
        while self.peek() is not None and self.peek() not in self.KEYWORDS and self.peek() not in self.SELECTORS:
            vals.append(self.take())
        if not vals:
            raise ValueError("selection keyword without values")
        return vals

    def atom(self):
        t = self.take()
        top = self.top
        n = top.n_atoms
        if t == "all":
            return np.ones(n, bool)
        if t == "none":
            return np.zeros(n, bool)
        if t == "protein":
            return np.array([r in PROTEIN_RESNAMES for r in top.resnames], bool)
        if t == "backbone":
            prot = np.array([r in PROTEIN_RESNAMES for r in top.resnames], bool)
            return prot & np.array([a in BACKBONE_NAMES for a in top.names], bool)
        if t in ("name", "resname"):
            pats = self._values()
            field = top.names if t == "name" else top.resnames
            return np.array([any(fnmatch.fnmatchcase(v, p) for p in pats) for v in field], bool)
        if t in ("resid", "index", "bynum"):
            field = top.resids if t == "resid" else np.arange(n) + (1 if t == "bynum" else 0)
            m = np.zeros(n, bool)
            for v in self._values():
                lo, hi = _range(v)
                m |= (field >= lo) & (field <= hi)
            return m
        raise ValueError(f"unsupported selection keyword {t!r} (native fallback; use MDAnalysis for the full language)")


def _range(v: str):
    for sep in ("-", ":"):
        if sep in v[1:]:
            a, b = v.split(sep, 1) if not v.startswith("-") else (v, v)
            return int(a), int(b)
    return int(v), int(v)


def write_gro(path: str, resids, resnames, names, frames_angstrom, box=(10.0, 10.0, 10.0), title="rmsf_amd"):
    """Write a (multi-frame) .gro file, %8.3f nm coordinates (tests/tools)."""
    frames = np.asarray(frames_angstrom, dtype=np.float32)
    if frames.ndim == 2:
        frames = frames[None]
    with open(path, "w") as fh:
        for f in frames:
            fh.write(f"{title}\n{len(names):5d}\n")
            for k, (ri, rn, an) in enumerate(zip(resids, resnames, names)):
                x, y, z = (f[k].astype(np.float64) / 10.0)
                fh.write(f"{int(ri) % 100000:5d}{rn:<5s}{an:>5s}{(k + 1) % 100000:5d}{x:8.3f}{y:8.3f}{z:8.3f}\n")
            fh.write("".join(f"{b:10.5f}" for b in box) + "\n")
