"""Host enqueue time of one RMSF step (run_pipeline) against its GPU time,
at the 8-GPU strong-scaling share (100k atoms x 2,500 frames, HBM-resident):
if the Python host side took longer than the kernels, an N-GPU run would be
host-bound.  Prints host us/step (no synchronisation inside the loop) and
wall us/step (synchronised).  Usage: python tools/time_host_step.py [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mdanalysis-mpi_amd"))
import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def main(nf=2500, n_atoms=100_000, steps=200):
    eng = Engine(torch.device("cuda", 0))
    for align in (None, "frame0", "average"):
        traj = generate(eng, n_atoms, 0, nf, seed=0, motion=motion_table(1, nf) if align else None)
        src = DeviceSource(traj)
        fl = FrameList(nf)
        for _ in range(5):
            run_pipeline(eng, src, fl, align=align)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run_pipeline(eng, src, fl, align=align)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"align={align}: host enqueue {1e6 * (t1 - t0) / steps:7.1f} us/step, "
              f"wall {1e6 * (t2 - t0) / steps:7.1f} us/step", flush=True)
        del traj, src
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
