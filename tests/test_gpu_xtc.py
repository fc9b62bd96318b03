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
