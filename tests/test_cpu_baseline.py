"""bench.py's CPU baseline leg (oracle/cpu_baseline.py): the multi-process
restatement of ``mpirun -n P python RMSF.py`` computes what the oracle's
in-process emulation computes, and sizes itself to the usable host cores."""
import os

import numpy as np
import pytest

from oracle import cpu_baseline as CB
from oracle import rmsf_oracle as O
from oracle import synth as SY
from rmsf_amd.synth import motion_table


def test_available_cores_respects_affinity():
    cores, aff, quota = CB.available_cores()
    assert aff == len(os.sched_getaffinity(0))
    assert 1 <= cores <= aff
    if quota is not None:
        assert cores == min(aff, quota)


@pytest.mark.parametrize("align", ["none", "frame0", "average"])
def test_baseline_matches_oracle_emulation(align):
    n_atoms, per, procs = 300, 5, 3
    mt = None if align == "none" else motion_table(1, per * procs)
    got = CB.run(n_atoms, per, procs=procs, align=align, motion=mt, want_rmsf=True)
    assert got["cores"] == procs and got["value"] > 0
    traj = SY.frames(0, n_atoms, 0, per * procs, mt)
    exp = O.rmsf_script(traj, None, None, size=procs, align=None if align == "none" else align)
    # same per-rank statements, same rank-order Chan fold: bit for bit
    np.testing.assert_array_equal(got["rmsf"], exp["rmsf"])
