"""Randomised parity sweep (not product code, not a test): random shapes,
selections, align modes, frame selections and inputs (HBM tensor / host
array in rows or coordinate planes / HBM planes / DCD or XTC file / one-process
gpus=1)
through RMSF(...).run() vs the oracle's RMSF.py
restatement on the selected frames; the unaligned cases also through
RMSF(..., exact=True), which must match the restatement bit for bit.  python tools/fuzz_parity.py [n_cases [--big]]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import rmsf_oracle as O  # noqa: E402
from oracle import synth as SY  # noqa: E402
from rmsf_amd import RMSF  # noqa: E402
from rmsf_amd.dcd import write_dcd  # noqa: E402
from rmsf_amd.xtc import XTCFile, write_xtc  # noqa: E402
from rmsf_amd.synth import motion_table  # noqa: E402


def main():
    n_cases = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(2026)
    worst, n_exact = 0.0, 0
    tmp = tempfile.mkdtemp(prefix="fuzz_")
    big = "--big" in sys.argv[2:]  # larger shapes: up to 200k atoms / 4,000 frames, <= 2e7 atom-frames
    for k in range(n_cases):
        na = int(rng.integers(1, 200_000 if big else 3000))
        nf = int(rng.integers(1, 4000 if big else 200))
        if big:
            nf = max(1, min(nf, 20_000_000 // na))
        traj = SY.frames(int(rng.integers(0, 1 << 30)), na, 0, nf, motion_table(int(rng.integers(0, 99)), nf))
        sel = np.sort(rng.choice(na, int(rng.integers(1, na + 1)), replace=False))
        align = [None, "frame0", "average"][int(rng.integers(0, 3))]
        frames = np.flatnonzero(rng.random(nf) < rng.uniform(0.2, 1.0))
        if frames.size == 0 or frames[0] != 0:
            frames = np.concatenate([[0], frames[frames != 0]])  # keep the frame-0 reference in the list
        where = ["device", "host", "soa", "dcd", "xtc", "gpus1", "dsoa"][int(rng.integers(0, 7))]
        kw = {}
        if where == "device":
            x = torch.tensor(traj, device="cuda")
        elif where in ("host", "gpus1"):
            x = traj
            if where == "gpus1":  # one process, the context ABI (rmsf_amd.multi)
                kw["gpus"] = 1
        elif where == "soa":  # [F, 3, n] coordinate planes, interleaved by the stager
            x = np.ascontiguousarray(traj.transpose(0, 2, 1))
            kw["layout"] = "soa"
        elif where == "dsoa":  # the same planes resident in HBM, read in place
            x = torch.tensor(np.ascontiguousarray(traj.transpose(0, 2, 1)), device="cuda")
            kw["layout"] = "soa"
        elif where == "dcd":
            x = os.path.join(tmp, f"c{k}.dcd")
            write_dcd(x, traj)
        else:  # XTC is lossy: the oracle sees the frames as the (host) codec reads them back
            x = os.path.join(tmp, f"c{k}.xtc")
            write_xtc(x, traj)
            with XTCFile(x) as f:
                traj = f.read()
        bf = int(rng.integers(1, 64))
        if big and rng.random() < 0.4:
            bf = None  # the whole block in one batch (HBM inputs: one launch per sweep)
        got = RMSF(x, select=sel, align=align, batch_frames=bf, **kw).run(frames=frames).results.rmsf
        exp = O.rmsf_script(traj[frames], sel, None, size=1, align=align)["rmsf"]
        # a one-atom superposition is undefined: NaN in qcprot (and the oracle) -- and on the device
        assert np.array_equal(np.isnan(got), np.isnan(exp)), f"case {k}: NaN pattern differs"
        ok = ~np.isnan(exp)
        err = float(np.abs(got[ok] - exp[ok]).max()) if ok.any() else 0.0
        worst = max(worst, err)
        print(f"case {k:2d}: {na:5d} atoms {len(sel):5d} sel {len(frames):4d}/{nf:3d} frames align={align} "
              f"{where:6s} batch={bf} max|d|={err:.2e}", flush=True)
        assert err < 1e-6, f"case {k}: {err}"
        if align is None and where != "gpus1":
            # exact=True: RMSF.py:120-146's own arithmetic, bit for bit
            ex = RMSF(x, select=sel, exact=True, batch_frames=bf, **kw).run(frames=frames).results.rmsf
            assert np.array_equal(ex.view(np.uint64), exp.view(np.uint64)), f"case {k}: exact=True differs"
            n_exact += 1
    print(f"all {n_cases} cases within 1e-6 A (worst {worst:.2e}); exact=True bit for bit in all {n_exact} "
          f"unaligned cases")


if __name__ == "__main__":
    main()
