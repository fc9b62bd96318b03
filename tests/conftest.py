"""pytest config: the ``gpu`` marker and import paths.

``-m "not gpu"`` runs everywhere (oracle vs golden vectors, host logic, the
C-ABI library's symbol table, gloo world_size-2 merges); ``-m gpu`` needs a
MI355X and exercises the HIP kernels through the C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mdanalysis-mpi_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
