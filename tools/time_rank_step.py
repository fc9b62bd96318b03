#!/usr/bin/env python3
"""Device time of one rank's C2 step at the strong-scaling shares
(100k atoms x 20k/N frames) on one GPU, with the N>1 merge's kernels in
place of the N=1 finalise: accumulate + fold, then the shift frame's gather,
k_chan_shift_pack and k_chan_shift_finish -- everything of an N-GPU step
but the all-reduce itself (and the broadcast beside the sweep), which needs
N devices.  Gives the per-rank floor of the N-GPU step time, i.e. an upper
bound on the strong-scaling efficiency the driver can measure.

  python tools/time_rank_step.py [--reps 30]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from rmsf_amd import parallel  # noqa: E402
from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import Accumulator, run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    eng = Engine(torch.device("cuda", 0))
    n_atoms, total = 100_000, 20_000
    traj = generate(eng, n_atoms, 0, total, seed=0)
    torch.cuda.synchronize()
    for n_gpus in (1, 2, 4, 8):
        nf = total // n_gpus
        shard = traj[:nf]
        src = DeviceSource(shard, n_traj=nf)
        fl = FrameList(nf)
        shift = torch.empty(3 * n_atoms, dtype=torch.float32, device=eng.device)

        def n1_step():  # the N=1 pipeline step: accumulate + fold + finalise
            run_pipeline(eng, src, fl)

        def rank_step():  # one rank of an N-GPU step, minus the collectives
            acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
            eng.gather_frames(shard.data_ptr(), shard.stride(0), eng.zero_index(), 1, n_atoms, None, shift)
            b = next(src.batches(fl, 0, nf, nf, eng.stream))
            acc.add(b)
            parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, nf, shift)

        row = {"n_gpus_share": n_gpus, "frames_per_gpu": nf}
        for name, fn in (("n1_step_ms", n1_step), ("rank_step_no_collective_ms", rank_step), ("n1_step_ms_again", n1_step)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):  # back to back, as bench.py's timed steps: device-bound
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10)
            ts.sort()
            row[name] = ts[len(ts) // 2]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
