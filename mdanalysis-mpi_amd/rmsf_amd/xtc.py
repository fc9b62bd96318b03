"""GROMACS XTC files through the native reader/writer (csrc/xtc.cpp).

``XTCFile`` replaces the libxdrfile-backed reader MDAnalysis uses for the
reference's GRO/XTC input (RMSF.py:34,56,92,124): frames are indexed once and
decoded frame-parallel on host threads, positions in Angstrom with
MDAnalysis' rounding.  ``write_xtc`` writes the same format (used by tests and
to produce inputs).  Host-only: no GPU needed.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import call


class XTCFile:
    def __init__(self, path: str):
        self.path = str(path)
        self._h = ctypes.c_void_p()
        na, nf = ctypes.c_int64(), ctypes.c_int64()
        call("rmsf_xtc_open", self.path.encode(), ctypes.byref(self._h), ctypes.byref(na), ctypes.byref(nf))
        self.n_atoms, self.n_frames = na.value, nf.value

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def __len__(self) -> int:
        return self.n_frames

    def read(self, start: int = 0, n: int | None = None, step: int = 1, sel=None, n_threads: int = 4) -> np.ndarray:
        """float32 [n, n_sel or n_atoms, 3] in Angstrom."""
        if n is None:
            n = len(range(start, self.n_frames, step))
        s = None if sel is None else np.ascontiguousarray(sel, dtype=np.int32)
        rows = self.n_atoms if s is None else len(s)
        out = np.empty((n, rows, 3), dtype=np.float32)
        call("rmsf_xtc_read", self._h, start, n, step, None if s is None else s.ctypes.data, rows,
             out.ctypes.data, n_threads)
        return out

    def frame_info(self, f: int):
        st, tm = ctypes.c_int32(), ctypes.c_float()
        box = np.empty(9, dtype=np.float32)
        call("rmsf_xtc_frame_info", self._h, f, ctypes.byref(st), ctypes.byref(tm), box.ctypes.data)
        return st.value, tm.value, box.reshape(3, 3)

    def record(self, f: int) -> tuple[int, int]:
        """(byte offset, byte length) of frame f's XDR record in the file."""
        off, n = ctypes.c_int64(), ctypes.c_int64()
        call("rmsf_xtc_frame_record", self._h, f, ctypes.byref(off), ctypes.byref(n))
        return off.value, n.value

    def close(self) -> None:
        if self._h:
            call("rmsf_xtc_close", self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_xtc(path: str, xyz: np.ndarray, precision: float = 1000.0, box=None, append: bool = False) -> None:
    """Write float32 [n_frames, n_atoms, 3] (Angstrom) as XTC."""
    x = np.ascontiguousarray(xyz, dtype=np.float32)
    if x.ndim == 2:
        x = x[None]
    b = None if box is None else np.ascontiguousarray(box, dtype=np.float32).reshape(9)
    call("rmsf_xtc_write", str(path).encode(), x.ctypes.data, x.shape[0], x.shape[1], float(precision),
         None if b is None else b.ctypes.data, int(append))
