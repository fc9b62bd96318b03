"""rmsf_amd -- MI355X-native frame-parallel RMSF (drop-in for the hot path of
i2nico/MDAnalysis-MPI ``RMSF.py``).

Public surface (mirrors the reference's names):
  * ``RMSF(atomgroup, align=...).run(start, stop, step).results.rmsf``
  * ``second_order_moments`` / ``get_rotation_matrix`` / ``CalcRMSDRotationalMatrix``
    (device-backed versions of RMSF.py:36-51 and MDAnalysis.lib.qcprot)
  * ``blocks`` -- the RMSF.py:65-69 frame decomposition
"""
from ._lib import RmsfEmptyError, RmsfError, load as load_library
from .parallel import blocks
from .qcprot import CalcRMSDRotationalMatrix, get_rotation_matrix
from .moments import second_order_moments
from .rms import RMSF, Results

__all__ = [
    "RMSF",
    "Results",
    "blocks",
    "second_order_moments",
    "get_rotation_matrix",
    "CalcRMSDRotationalMatrix",
    "RmsfError",
    "RmsfEmptyError",
    "load_library",
]
