#!/usr/bin/env python3
"""Device time of one rank's C2 step at the strong-scaling shares
(100k atoms x 20k/N frames) on one GPU, with the N>1 merge's kernels in
place of the N=1 finalise: accumulate + fold, then the shift frame's gather,
k_chan_shift_pack and k_chan_shift_finish -- everything of an N-GPU step
but the all-reduce itself (and the broadcast beside the sweep), which needs
N devices.  Three forms: the round-2 step (fold, then a pack launch), the
pipeline's step (the last fold writes the packed moments,
rmsf_fold_balanced_shift), and that step captured as a hipGraph; all three
must give bit-identical results.  "of_perfect_split" = (N=1 step / N) / the
rank step.  Gives the per-rank floor of the N-GPU step time, i.e. an upper
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
    ap.add_argument("--shares", type=int, nargs="*", default=[1, 2, 4, 8], help="N of the N-GPU shares to time")
    a = ap.parse_args()
    eng = Engine(torch.device("cuda", 0))
    n_atoms, total = 100_000, 20_000
    traj = generate(eng, n_atoms, 0, total, seed=0)
    torch.cuda.synchronize()
    base = None
    for n_gpus in a.shares:
        nf = total // n_gpus
        shard = traj[:nf]
        src = DeviceSource(shard, n_traj=nf)
        fl = FrameList(nf)
        shift = torch.empty(3 * n_atoms, dtype=torch.float32, device=eng.device)

        def n1_step():  # the N=1 pipeline step: accumulate + fold + finalise
            run_pipeline(eng, src, fl)

        def rank_step_unfused():  # one rank of an N-GPU step, minus the collectives (round 2 form)
            acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
            eng.gather_frames(shard.data_ptr(), shard.stride(0), eng.zero_index(), 1, n_atoms, None, shift)
            b = next(src.batches(fl, 0, nf, nf, eng.stream))
            acc.add(b)
            return parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, nf, shift)

        t = torch.empty(6 * n_atoms, dtype=torch.float64, device=eng.device)
        acc_g = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)

        def rank_step(acc=None):  # the pipeline's form: the last fold packs the merge's moments
            if acc is None:
                acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
            acc.n, acc.packed = 0, False
            eng.gather_frames(shard.data_ptr(), shard.stride(0), eng.zero_index(), 1, n_atoms, None, shift)
            b = next(src.batches(fl, 0, nf, nf, eng.stream))
            acc.add(b, pack=(shift, None, t, None))
            assert acc.packed
            return parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, nf, shift, packed=t)

        def rank_step_side(acc=None):  # as run_pipeline: the shift's gather on a side stream beside the sweep
            if acc is None:
                acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
            acc.n, acc.packed = 0, False
            main = torch.cuda.current_stream(eng.device)
            side = eng.side_stream
            side.wait_stream(main)
            with torch.cuda.stream(side):
                eng.gather_frames(shard.data_ptr(), shard.stride(0), eng.zero_index(), 1, n_atoms, None, shift)
                ev = torch.cuda.Event()
                ev.record(side)

            class _Wait:  # what parallel.broadcast_async's work does at N=1 size
                def wait(self):
                    main.wait_event(ev)
            b = next(src.batches(fl, 0, nf, nf, eng.stream))
            acc.add(b, pack=(shift, None, t, _Wait()))
            return parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, nf, shift, packed=t)

        # the same step recorded once as a hipGraph and replayed
        side = torch.cuda.Stream(eng.device)
        side.wait_stream(torch.cuda.current_stream(eng.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                rank_step(acc_g)
        torch.cuda.current_stream(eng.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = rank_step(acc_g)
        torch.cuda.synchronize()

        def rank_step_graph():
            graph.replay()
            return g_out

        # bit-identity of the three forms
        r_u, r_f = rank_step_unfused(), rank_step()
        r_s = [x.clone() for x in rank_step_side()]
        graph.replay()
        torch.cuda.synchronize()
        same = all(all(torch.equal(x, y) for x, y in zip(r_u, r)) for r in (r_f, r_s, g_out))

        row = {"n_gpus_share": n_gpus, "frames_per_gpu": nf, "fused_and_graph_bitwise_equal_unfused": bool(same)}
        for name, fn in (("n1_step_ms", n1_step), ("rank_step_unfused_ms", rank_step_unfused),
                         ("rank_step_fused_ms", rank_step), ("rank_step_fused_graph_ms", rank_step_graph),
                         ("rank_step_fused_side_gather_ms", rank_step_side),
                         ("n1_step_ms_again", n1_step)):
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
        if n_gpus == 1:
            base = row["n1_step_ms"]
        if base is not None:
            perfect = base / n_gpus
            for k in ("rank_step_unfused_ms", "rank_step_fused_ms", "rank_step_fused_graph_ms",
                      "rank_step_fused_side_gather_ms"):
                row[k.replace("_ms", "_of_perfect_split")] = perfect / row[k]
        print(json.dumps(row), flush=True)
        del graph


if __name__ == "__main__":
    main()
