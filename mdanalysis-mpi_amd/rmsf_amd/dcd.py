"""CHARMM / NAMD / X-PLOR DCD trajectories (BASELINE config C1's adk PSF/DCD).

MDAnalysis reads DCD with its bundled ``libdcd``; RMSF.py reaches it through
``universe.trajectory[frame]`` (RMSF.py:92,124) when the Universe is built
from a PSF/DCD pair.  A DCD file is Fortran-unformatted binary: every record
is framed by its byte length (int32).  Header records:

  84 | "CORD" | int32 ICNTRL[20] | 84        NSET = ICNTRL[0] frames,
                                              NAMNF = ICNTRL[8] fixed atoms,
                                              CHARMM files: ICNTRL[19] != 0,
                                              unit-cell flag ICNTRL[10],
                                              4D flag ICNTRL[11]
  title record (int32 NTITLE, NTITLE x 80 bytes)
  4 | NATOM | 4
  free-atom indices (1-based, NATOM - NAMNF of them) if NAMNF > 0

and per frame: [unit cell: 6 float64, CHARMM with the flag] then the X, Y
and Z records (float32, Angstrom -- MDAnalysis applies no conversion) and,
for 4D CHARMM files, a W record.  Frame 0 stores every atom; with fixed
atoms the later frames store only the free ones, the fixed ones keep frame
0's coordinates.  Byte order is detected from the first marker.

Host-only numpy (the files are raw float32 planes, memory-mapped; frames are
interleaved to the (frame, atom, xyz) layout the GPU path streams).  The
format is restated from its published description; no DCD file exists in
this environment, so it is pinned by a write -> read round trip and an
independent record-by-record parse in the tests (``format unpinned`` as for
XTC).
"""
from __future__ import annotations

import os

import numpy as np


class DCDFile:
    def __init__(self, path: str):
        self.path = os.fspath(path)
        raw = np.memmap(self.path, dtype=np.uint8, mode="r")
        if raw.size < 92:
            raise ValueError(f"{self.path}: too short for a DCD header")
        first_le = int(np.frombuffer(raw[:4].tobytes(), "<i4")[0])
        first_be = int(np.frombuffer(raw[:4].tobytes(), ">i4")[0])
        if first_le == 84:
            self._e = "<"
        elif first_be == 84:
            self._e = ">"
        else:
            raise ValueError(f"{self.path}: not a DCD file (first record marker is not 84)")
        if raw[4:8].tobytes() != b"CORD":
            raise ValueError(f"{self.path}: missing 'CORD' signature")
        e = self._e
        i4 = np.dtype(e + "i4")
        icntrl = np.frombuffer(raw[8:88].tobytes(), i4)
        self._check(raw, 88, 84)
        self.charmm = int(icntrl[19]) != 0
        self.has_cell = self.charmm and int(icntrl[10]) != 0
        self.has_4d = self.charmm and int(icntrl[11]) != 0
        namnf = int(icntrl[8])
        pos = 92
        tlen = self._marker(raw, pos)
        pos += 4 + tlen
        self._check(raw, pos, tlen)
        pos += 4
        if self._marker(raw, pos) != 4:
            raise ValueError(f"{self.path}: bad NATOM record")
        self.n_atoms = int(np.frombuffer(raw[pos + 4:pos + 8].tobytes(), i4)[0])
        self._check(raw, pos + 8, 4)
        pos += 12
        self.free = None
        if namnf > 0:
            nfree = self.n_atoms - namnf
            if self._marker(raw, pos) != 4 * nfree:
                raise ValueError(f"{self.path}: bad free-atom record")
            self.free = np.frombuffer(raw[pos + 4:pos + 4 + 4 * nfree].tobytes(), i4).astype(np.int64) - 1
            self._check(raw, pos + 4 + 4 * nfree, 4 * nfree)
            pos += 8 + 4 * nfree
        self._raw = raw
        self._data0 = pos
        self._full = self._frame_bytes(self.n_atoms)
        self._rest = self._frame_bytes(self.n_atoms if self.free is None else len(self.free))
        body = raw.size - pos
        self.n_frames = 0 if body < self._full else 1 + (body - self._full) // self._rest
        if self.n_frames and icntrl[0] > 0 and int(icntrl[0]) != self.n_frames:
            # NSET is not always maintained by writers; MDAnalysis trusts the file size as well
            pass

    def _marker(self, raw, pos: int) -> int:
        return int(np.frombuffer(raw[pos:pos + 4].tobytes(), self._e + "i4")[0])

    def _check(self, raw, pos: int, want: int) -> None:
        if self._marker(raw, pos) != want:
            raise ValueError(f"{self.path}: record length markers disagree at byte {pos}")

    def _frame_bytes(self, n: int) -> int:
        planes = 4 if self.has_4d else 3
        return (56 if self.has_cell else 0) + planes * (8 + 4 * n)

    def _frame(self, f: int) -> np.ndarray:
        """float32 [n_atoms, 3] of frame f (fixed atoms from frame 0)."""
        if not 0 <= f < self.n_frames:
            raise IndexError(f"frame {f} out of range ({self.n_frames} frames)")
        full = f == 0 or self.free is None
        n = self.n_atoms if full else len(self.free)
        off = self._data0 + (0 if f == 0 else self._full + (f - 1) * self._rest)
        if self.has_cell:
            off += 56
        out = np.empty((self.n_atoms, 3), dtype=np.float32)
        if not full:
            out[:] = self._frame(0)
        f4 = np.dtype(self._e + "f4")
        for c in range(3):
            if self._marker(self._raw, off) != 4 * n:
                raise ValueError(f"{self.path}: frame {f}: bad coordinate record")
            v = np.frombuffer(self._raw[off + 4:off + 4 + 4 * n].tobytes(), f4)
            if full:
                out[:, c] = v
            else:
                out[self.free, c] = v
            off += 8 + 4 * n
        return out

    def read(self, start: int = 0, n: int | None = None, step: int = 1, sel=None) -> np.ndarray:
        """float32 [n, n_sel or n_atoms, 3] in Angstrom."""
        frames = range(start, self.n_frames, step)
        if n is not None:
            frames = frames[:n]
        idx = None if sel is None else np.asarray(sel, dtype=np.int64)
        rows = self.n_atoms if idx is None else len(idx)
        out = np.empty((len(frames), rows, 3), dtype=np.float32)
        if self.free is None and not self.has_4d:
            # fixed-size frames: one strided view of the whole file
            e = self._e
            n_at = self.n_atoms
            fields = ([("cm0", e + "i4"), ("cell", e + "f8", (6,)), ("cm1", e + "i4")] if self.has_cell else [])
            for c in "xyz":
                fields += [(f"m0{c}", e + "i4"), (c, e + "f4", (n_at,)), (f"m1{c}", e + "i4")]
            rec = np.ndarray((self.n_frames,), dtype=np.dtype(fields), buffer=self._raw, offset=self._data0)
            sub = rec[start::step][:len(frames)]
            for k, c in enumerate("xyz"):
                if np.any(sub[f"m0{c}"] != 4 * n_at):
                    raise ValueError(f"{self.path}: bad coordinate record markers")
                plane = sub[c]
                out[:, :, k] = plane if idx is None else plane[:, idx]
            return out
        for k, f in enumerate(frames):
            fr = self._frame(f)
            out[k] = fr if idx is None else fr[idx]
        return out

    def plane_ptrs(self, frames) -> tuple[np.ndarray, int] | None:
        """Host addresses of the X records of ``frames`` and the distance
        between a frame's X, Y and Z records in floats (4 n_atoms + 8 bytes),
        for staging the coordinate planes straight from the memory map
        (rmsf_stager_stage_planes interleaves them): native-endian files
        with every atom in every frame and no 4D record; otherwise None.
        Checks every frame's X/Y/Z record markers, as read() does."""
        import sys

        if self._e != ("<" if sys.byteorder == "little" else ">") or self.free is not None or self.has_4d:
            return None
        f = np.asarray(frames, dtype=np.int64)
        if f.size and (f.min() < 0 or f.max() >= self.n_frames):
            raise IndexError(f"frame out of range ({self.n_frames} frames)")
        n = self.n_atoms
        x0 = self._data0 + f * self._full + (56 if self.has_cell else 0)  # marker before the X record
        words = np.frombuffer(self._raw, dtype=np.int32, count=self._raw.size // 4)
        for k in range(3):
            m = x0 + k * (8 + 4 * n)
            if np.any(words[m // 4] != 4 * n) or np.any(words[(m + 4 + 4 * n) // 4] != 4 * n):
                raise ValueError(f"{self.path}: bad coordinate record markers")
        return (self._raw.ctypes.data + x0 + 4).astype(np.uint64), n + 2

    def close(self) -> None:
        self._raw = None

    def __len__(self) -> int:
        return self.n_frames

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_dcd(path: str, xyz: np.ndarray, box=None, charmm: bool = True, fixed=None, title: str = "rmsf_amd",
              byteorder: str = "<") -> None:
    """Write float32 [n_frames, n_atoms, 3] (Angstrom) as a DCD file.

    ``box``: 6 floats written as each frame's unit-cell record (CHARMM only).
    ``fixed``: atom indices held fixed (stored in frame 0 only)."""
    x = np.ascontiguousarray(xyz, dtype=np.float32)
    if x.ndim == 2:
        x = x[None]
    nf, na, _ = x.shape
    e = byteorder
    fixed = np.zeros(0, np.int64) if fixed is None else np.unique(np.asarray(fixed, dtype=np.int64))
    free = np.setdiff1d(np.arange(na), fixed)
    icntrl = np.zeros(20, dtype=e + "i4")
    icntrl[0], icntrl[1], icntrl[2], icntrl[3] = nf, 0, 1, nf
    icntrl[8] = len(fixed)
    if charmm:
        icntrl[9] = np.array([1.0], dtype=e + "f4").view(e + "i4")[0]
        icntrl[10] = 1 if box is not None else 0
        icntrl[19] = 24
    i4 = lambda v: np.array([v], dtype=e + "i4").tobytes()  # noqa: E731
    with open(path, "wb") as fh:
        fh.write(i4(84) + b"CORD" + icntrl.tobytes() + i4(84))
        t = title.encode()[:80].ljust(80)
        fh.write(i4(84) + i4(1) + t + i4(84))
        fh.write(i4(4) + i4(na) + i4(4))
        if len(fixed):
            fh.write(i4(4 * len(free)) + (free + 1).astype(e + "i4").tobytes() + i4(4 * len(free)))
        for f in range(nf):
            if charmm and box is not None:
                fh.write(i4(48) + np.asarray(box, dtype=e + "f8").tobytes() + i4(48))
            rows = np.arange(na) if (f == 0 or not len(fixed)) else free
            for c in range(3):
                v = x[f, rows, c].astype(e + "f4")
                fh.write(i4(4 * len(rows)) + v.tobytes() + i4(4 * len(rows)))
