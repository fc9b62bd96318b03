"""CPU tier: argument checks of the SoA (coordinate-plane) host input that
run before any device work (the staging itself is GPU-tier,
tests/test_gpu_soa.py)."""
import numpy as np
import pytest

from rmsf_amd import RMSF


def test_layout_values():
    x = np.zeros((2, 3, 5), np.float32)
    RMSF(x, layout="soa")
    RMSF(x.transpose(0, 2, 1), layout="fac")
    with pytest.raises(ValueError, match="layout"):
        RMSF(x, layout="aos")


@pytest.mark.parametrize("inp", ["traj.xtc", "traj.dcd", object()])
def test_soa_only_for_arrays(inp):
    with pytest.raises(ValueError, match="numpy array or HIP tensor"):
        RMSF(inp, layout="soa")
