#!/usr/bin/env python3
"""The one-process multi-context step against the torchrun rank step, on one GPU.

At a strong-scaling share (100k atoms x 20k/N frames) it times, in one
process, 10 back-to-back steps (wall clock, synchronised at the end) of:

  pipeline_rank_step   the torchrun form's rank step minus the collectives
                       (tools/time_rank_step.py's "fused, side gather":
                       accumulate, the fold that packs T1/T2, unpack+finish;
                       the shift frame gathered on a side stream)
  context_step_1       ONE context doing the one-process form's step:
                       rmsf_multi_push_frames (reset, shift frame, push) +
                       rmsf_multi_chan_merge_root(root=0) with the no-op
                       transport -- the same kernels as the rank step
  context_step_N       N contexts all on device 0 (no-op transport): the
                       device work is N shares, so the wall clock is ~N x;
                       what it measures is the HOST side -- the enqueue time
                       of a whole step for N contexts with the device idle
                       (host_enqueue_ms), which must stay below one share's
                       device time for N real devices to run device-bound
                       ("host_in_loop" also counts the merge's wait for the
                       shift frame's digest, i.e. for the previous step;
                       on one GPU the 2N streams share 4 hardware queues, so
                       a digest can queue behind another context's sweep)
  context_step_N_tiny  the same over 8-frame blocks: the device work is
                       negligible, so the call time is the host cost alone

and checks that context_step_1 and the pipeline rank step give the same
RMSF bit for bit (same kernels, same shift, same order).

  python tools/time_multi_step.py [--share 8] [--contexts 8] [--reps 7]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from rmsf_amd import parallel  # noqa: E402
from rmsf_amd._lib import RMSF_MODE_WELFORD  # noqa: E402
from rmsf_amd.context import PUSH_WELFORD, TRANSPORT_NOOP, Context  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import Accumulator  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def idle_host(fn, sync, reps, inner=10):
    """Host time of one step call with the device idle (synchronised before
    each call): the pure enqueue cost, without waits on earlier steps."""
    hs = []
    for _ in range(reps * inner):
        sync()
        h0 = time.perf_counter()
        fn()
        hs.append((time.perf_counter() - h0) * 1e3)
    sync()
    hs.sort()
    return hs[len(hs) // 2]


def wall(fn, sync, reps, inner=10):
    for _ in range(3):
        fn()
    sync()
    ts, hs = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        h = 0.0
        for _ in range(inner):
            h0 = time.perf_counter()
            fn()
            h += time.perf_counter() - h0
        sync()
        ts.append((time.perf_counter() - t0) / inner * 1e3)
        hs.append(h / inner * 1e3)
    ts.sort()
    hs.sort()
    return ts[len(ts) // 2], hs[len(hs) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share", type=int, default=8, help="N of the 100k x 20k/N share")
    ap.add_argument("--contexts", type=int, default=8)
    ap.add_argument("--n-atoms", type=int, default=100_000)
    ap.add_argument("--total", type=int, default=20_000)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    eng = Engine(torch.device("cuda", 0))
    n_atoms, nf = a.n_atoms, a.total // a.share
    shard = generate(eng, n_atoms, 0, nf, seed=0)
    torch.cuda.synchronize()
    src = DeviceSource(shard, n_traj=nf)
    fl = FrameList(nf)
    shift = torch.empty(3 * n_atoms, dtype=torch.float32, device=eng.device)
    t = torch.empty(6 * n_atoms, dtype=torch.float64, device=eng.device)

    def rank_step():  # the pipeline's N>1 rank step minus the collectives (side-stream gather)
        acc = Accumulator(eng, n_atoms, RMSF_MODE_WELFORD, nf, False)
        main_s = torch.cuda.current_stream(eng.device)
        side = eng.side_stream
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            eng.gather_frames(shard.data_ptr(), shard.stride(0), eng.zero_index(), 1, n_atoms, None, shift)
            ev = torch.cuda.Event()
            ev.record(side)

        class _Wait:
            def wait(self):
                main_s.wait_event(ev)
        b = next(src.batches(fl, 0, nf, nf, eng.stream))
        acc.add(b, pack=(shift, None, t, _Wait()))
        return parallel.global_chan_shifted(eng, acc.result0, acc.result1, acc.n, nf, shift, packed=t)

    one = [Context(n_atoms, device=0)]
    Context.multi_set_transport(one, TRANSPORT_NOOP)
    frame0 = shard[0]

    def ctx_step(ctxs, blocks):
        Context.multi_push_frames(ctxs, blocks, PUSH_WELFORD, shift_frames=[frame0] * len(ctxs), after_torch=False)
        Context.multi_chan_merge(ctxs, root=0)

    def sync_ctxs(ctxs):
        def f():
            for c in ctxs:
                c.synchronize()
        return f

    # bit-identity: one context's step vs the pipeline rank step
    r_pipe = rank_step()[2].cpu().numpy()
    ctx_step(one, [shard])
    r_ctx = one[0].rmsf()
    row = {"n_atoms": n_atoms, "frames_per_share": nf, "share_of": a.share,
           "context_equals_pipeline_bitwise": bool((r_pipe == r_ctx).all()),
           "max_abs_diff": float(abs(r_pipe - r_ctx).max())}
    order = [("pipeline_rank_step", lambda: rank_step(), torch.cuda.synchronize),
             ("context_step_1", lambda: ctx_step(one, [shard]), sync_ctxs(one))]
    many = [Context(n_atoms, device=0) for _ in range(a.contexts)]
    Context.multi_set_transport(many, TRANSPORT_NOOP)
    order.append((f"context_step_{a.contexts}", lambda: ctx_step(many, [shard] * a.contexts), sync_ctxs(many)))
    order.append(("pipeline_rank_step_again", lambda: rank_step(), torch.cuda.synchronize))
    order.append(("context_step_1_again", lambda: ctx_step(one, [shard]), sync_ctxs(one)))
    for name, fn, sync in order:
        w, h = wall(fn, sync, a.reps)
        i = idle_host(fn, sync, a.reps)
        row[name + "_ms"] = w
        row[name + "_host_in_loop_ms"] = h      # includes waits on the previous step (host runs ~1 step ahead)
        row[name + "_host_enqueue_ms"] = i      # the call alone, device idle
        print(f"  {name}: {w:.4f} ms/step wall; host {h:.4f} ms/step in the loop, {i:.4f} ms with the device idle",
              file=sys.stderr, flush=True)
    # the host cost alone: N contexts over TINY blocks (8 frames each), so the
    # device work (and the queues 2N streams share on one GPU) cannot hold the
    # host up; with N real devices this is what the host adds per step
    tiny = shard[:8]
    w, h = wall(lambda: ctx_step(many, [tiny] * a.contexts), sync_ctxs(many), a.reps)
    row[f"context_step_{a.contexts}_tiny_ms"] = w
    row[f"context_step_{a.contexts}_tiny_host_enqueue_ms"] = idle_host(lambda: ctx_step(many, [tiny] * a.contexts),
                                                                       sync_ctxs(many), a.reps)
    # the same host cost split into the push call and the merge call
    sync_many = sync_ctxs(many)
    # (the merge call first waits for the shift frames' digests: on ONE device
    # the 2N streams share 4 hardware queues, so that wait is device time;
    # "merge_call_ready" times the merge with the pushes already finished --
    # its host cost alone)
    push_ms, merge_ms, ready_ms = [], [], []
    for _ in range(a.reps * 10):
        sync_many()
        h0 = time.perf_counter()
        Context.multi_push_frames(many, [tiny] * a.contexts, PUSH_WELFORD, shift_frames=[frame0] * a.contexts,
                                  after_torch=False)
        h1 = time.perf_counter()
        Context.multi_chan_merge(many, root=0)
        h2 = time.perf_counter()
        push_ms.append((h1 - h0) * 1e3)
        merge_ms.append((h2 - h1) * 1e3)
        sync_many()
        Context.multi_push_frames(many, [tiny] * a.contexts, PUSH_WELFORD, shift_frames=[frame0] * a.contexts,
                                  after_torch=False)
        sync_many()
        h3 = time.perf_counter()
        Context.multi_chan_merge(many, root=0)
        ready_ms.append((time.perf_counter() - h3) * 1e3)
    sync_many()
    for v in (push_ms, merge_ms, ready_ms):
        v.sort()
    row[f"context_step_{a.contexts}_tiny_push_call_ms"] = push_ms[len(push_ms) // 2]
    row[f"context_step_{a.contexts}_tiny_merge_call_ms"] = merge_ms[len(merge_ms) // 2]
    row[f"context_step_{a.contexts}_tiny_merge_call_ready_ms"] = ready_ms[len(ready_ms) // 2]
    w1, _ = wall(lambda: ctx_step(one, [tiny]), sync_ctxs(one), a.reps)
    row["context_step_1_tiny_ms"] = w1
    row["context_step_1_tiny_host_enqueue_ms"] = idle_host(lambda: ctx_step(one, [tiny]), sync_ctxs(one), a.reps)
    print(f"  tiny blocks: {a.contexts} contexts {w:.4f} ms/step wall, "
          f"{row[f'context_step_{a.contexts}_tiny_host_enqueue_ms']:.4f} ms host; 1 context {w1:.4f} ms wall, "
          f"{row['context_step_1_tiny_host_enqueue_ms']:.4f} ms host", file=sys.stderr, flush=True)
    p = min(row["pipeline_rank_step_ms"], row["pipeline_rank_step_again_ms"])
    c1 = min(row["context_step_1_ms"], row["context_step_1_again_ms"])
    row["context_1_over_pipeline"] = c1 / p
    row[f"context_{a.contexts}_tiny_host_over_share_step"] = row[f"context_step_{a.contexts}_tiny_host_enqueue_ms"] / p
    print(json.dumps(row), flush=True)
    for c in one + many:
        c.close()


if __name__ == "__main__":
    main()
