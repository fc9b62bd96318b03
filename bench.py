#!/usr/bin/env python3
"""Headline benchmark: atom-frames/s of the frame-parallel RMSF path on MI355X.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One "step" = one full RMSF pass of the hot path over the trajectory (the
per-frame Welford accumulator over every frame of each device's block, the
in-GPU Chan merge of the frame tiles, the cross-GPU Chan merge over RCCL,
the finalise), with the synthetic trajectory already resident in HBM.

Scaling (``--scaling``):
  strong (default)  ONE trajectory of ``--frames`` frames (c2: 100k atoms x
                    20k frames, BASELINE.json configs[1]; the north star's
                    "100k-atom x 20k-frame data at 1, 2, 4 and 8 GPUs") split
                    into the RMSF.py:65-69 frame blocks, one per GPU;
  weak              every GPU holds a ``--frames``-frame block (c4: 1M atoms x
                    2.5k frames per GPU = configs[3] at N=8).

Multi-GPU, two launch forms with the same arithmetic:
  * under torch.distributed.run (WORLD_SIZE set): one process per GPU,
    merges over torch.distributed's RCCL backend;
  * ``python bench.py --gpus N`` with no launcher: ONE process drives N
    devices through the C ABI's contexts (ncclCommInitAll, one
    stream per device, one host thread per device).  With fewer than N
    devices visible it fails, unless ``--rehearse`` (device 0 listed N
    times, in-process fold instead of RCCL; labelled in the output).

At N=1 the aligned configurations are measured too ("modes": C3 = QCP
alignment to frame 0; RMSF.py's own two-sweep "average").  Rank 0 prints ONE
JSON line.  ``roofline`` = algorithmic bytes (12 B per atom-frame, SURVEY
8(d)) of every timed launch of the dominant kernel / their summed duration,
from HIP events recorded around each launch on its own stream;
``cpu_baseline`` = the oracle's numpy restatement of RMSF.py's two sweeps on
the host's usable cores (``mpirun -n <cores> python RMSF.py`` shape), run
before the GPU is touched, with the unaligned (C2) sweep as a second figure.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md, chip table)
FP64_PEAK_TFS = 78.6    # MI355X fp64 vector spec (not in the local guide, unverified)
B_PER_ATOM_FRAME = 12   # algorithmic bytes per (atom, frame) per sweep
FLOP_PER_ATOM_FRAME_SUPERPOSE = 27  # covariance 18 + |x|^2 6 + COM 3
METRIC = "atom-frames/sec (RMSF) + achieved HBM GB/s fraction"

WORKLOADS = {
    "c2": dict(n_atoms=100_000, frames=20_000, align=None,
               name="C2: synthetic 100k atoms x 20k frames fp32, no alignment, fp64 Welford"),
    "c3": dict(n_atoms=100_000, frames=20_000, align="frame0",
               name="C3: synthetic 100k atoms x 20k frames fp32, QCP alignment to frame 0"),
    "average": dict(n_atoms=100_000, frames=20_000, align="average",
                    name="RMSF.py two-sweep: 100k atoms x 20k frames, align to frame 0, average, re-align"),
    "c4": dict(n_atoms=1_000_000, frames=2_500, align=None, scaling="weak",
               name="C4 share: synthetic 1M atoms x 2.5k frames fp32 per GPU (N=8: 1M x 20k, 240 GB)"),
    "c5": dict(n_atoms=250_000, frames=1_000, align=None, host=True,
               name="C5 (pre-decoded): 250k atoms x 1k frames fp32 in host memory, streamed via the pinned "
                    "multi-buffer stager (PCIe-inclusive rate; no XTC decode)"),
    "c5xtc": dict(n_atoms=250_000, frames=2048, align=None, host=True, xtc=True,
                  name="C5: 250k-atom XTC file (precision 1000) streamed from the host and decoded "
                       "(--xtc-decode gpu: compressed records via pinned slots, decompressed on the GPU; host: "
                       "decoded on host threads into the pinned stager); read + PCIe + decode inclusive"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="strong: --frames in total split over the GPUs (default); weak: --frames per GPU")
    ap.add_argument("--n-atoms", type=int, default=None)
    ap.add_argument("--frames", type=int, default=None,
                    help="trajectory frames (strong) or frames per GPU (weak); default: the workload's")
    ap.add_argument("--frames-per-gpu", type=int, default=None, help="shorthand for --scaling weak --frames F")
    ap.add_argument("--one-process", action="store_true",
                    help="the one-process context form (main_single_process) even at --gpus 1: one device "
                         "context, a one-rank ncclCommInitAll communicator")
    ap.add_argument("--rehearse", action="store_true",
                    help="one-process --gpus N with fewer devices: list device 0 N times (rehearsal)")
    ap.add_argument("--rehearse-transport", choices=["fold", "noop"], default="fold",
                    help="--rehearse: exchanges by the in-process host fold (exact, synchronising) or by a no-op "
                         "(host-cost timing only: the merged result is not the global one)")
    ap.add_argument("--splits", type=int, default=None)
    ap.add_argument("--batch-frames", type=int, default=None, help="aligned modes: frames per superpose batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=640,
                    help="frames per CPU process for the unaligned (C2) baseline sample")
    ap.add_argument("--cpu-average-frames", type=int, default=128,
                    help="frames per CPU process for the RMSF.py two-sweep baseline sample")
    ap.add_argument("--no-modes", action="store_true", help="skip the aligned-mode measurements at N=1")
    ap.add_argument("--mode-steps", type=int, default=3)
    ap.add_argument("--mode-warmup", type=int, default=3,
                    help="untimed steps before each mode's timed steps (the first 2-3 exact runs of a fresh "
                         "process are 5-15 %% slower: tools/probe_seq_bench.py)")
    ap.add_argument("--no-io-modes", action="store_true",
                    help="N=1: skip the C4-share and C5-XTC modes (30 GB of frames, a 2.7 GB XTC file)")
    ap.add_argument("--stager-threads", type=int, default=4)
    ap.add_argument("--stager-batch", type=int, default=None, help="c5: frames per staged batch")
    ap.add_argument("--xtc-decode", choices=["gpu", "host"], default="gpu",
                    help="c5xtc: decompress the XTC records on the GPU (default) or on host threads")
    ap.add_argument("--xtc-cache", action="store_true",
                    help="c5xtc (GPU decode): keep decoded frames in HBM within a step (RMSF.py's second sweep "
                         "reads them from HBM); dropped before every step, so each step decodes once")
    ap.add_argument("--host-layout", choices=["fac", "soa"], default="fac",
                    help="c5: the host array as [F, n_atoms, 3] (fac) or as x/y/z coordinate planes [F, 3, n_atoms] "
                         "(soa: the stager interleaves them on the host)")
    ap.add_argument("--host-cache", action="store_true",
                    help="c5: keep the staged frames in HBM within a step (RMSF.py's second sweep reads them there)")
    ap.add_argument("--align", choices=["none", "frame0", "average"], default=None, help="override the workload's")
    ap.add_argument("--merge-slabs", type=int, default=None,
                    help="N>1, no alignment: atom slabs of the final sweep whose all-reduces overlap the next slab "
                         "(default: 2 from 1M atoms, else none; 0 = off)")
    ap.add_argument("--merge", choices=["root", "all", "scatter"], default="root",
                    help="N>1: the final Chan merge as a reduce to rank 0 (default: RMSF.py:143's "
                         "comm.reduce(root=0); a ring reduce carries the 6*n_sel doubles over each link once), as "
                         "an all-reduce that leaves the result on every rank (twice the link bytes), or as a "
                         "reduce-scatter by atom slices with each rank finishing its slice and only the RMSF "
                         "gathered to rank 0 (torchrun form; the one-process form treats it as root)")
    ap.add_argument("--merge-root", action="store_const", dest="merge", const="root",
                    help="same as --merge root (kept for older command lines)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL; gloo only "
                                                     "to rehearse several ranks on one GPU)")
    return ap.parse_args(argv)


def resolve(a, world: int) -> dict:
    """The workload of this run: atoms, frames in total, this run's scaling."""
    wl = dict(WORKLOADS[a.workload])
    if a.n_atoms:
        wl["n_atoms"] = a.n_atoms
    scaling = a.scaling or wl.get("scaling", "strong")
    frames = wl["frames"]
    if a.frames_per_gpu:
        scaling, frames = "weak", a.frames_per_gpu
    if a.frames:
        frames = a.frames
    if a.align is not None:
        wl["align"] = None if a.align == "none" else a.align
    wl["scaling"] = scaling
    wl["n_total"] = frames * world if scaling == "weak" else frames
    if wl["n_total"] < world:
        raise SystemExit(f"{wl['n_total']} frames cannot give each of {world} GPUs a block")
    return wl


def device_plan(n: int, visible: int, rehearse: bool) -> tuple[list[int], bool]:
    """Devices for a one-process ``--gpus n`` run: 0..n-1, or (``rehearse``)
    device 0 listed n times when fewer are visible.  Fails loudly otherwise."""
    if n < 1:
        raise SystemExit("--gpus must be >= 1")
    if visible >= n:
        return list(range(n)), False
    if rehearse and visible >= 1:
        return [0] * n, True
    raise SystemExit(f"--gpus {n} asks for {n} devices but {visible} are visible "
                     f"(launch under torch.distributed.run on an {n}-GPU node, or pass --rehearse "
                     f"to run {n} device contexts on device 0)")


def load_traffic(workload: str, n_atoms: int, n_frames: int):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    summary (profiles/pmc_<workload>.json, written by tools/pmc_summary.py
    from separate rocprofv3 --pmc passes), if one exists for this shape."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("n_atoms") == n_atoms and d.get("n_frames") == n_frames:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def roofline(kernel: str, launches: int, ms: float, atom_frames: float, traffic=None, traffic_source=None) -> dict:
    """Algorithmic bytes of the timed launches over their summed duration."""
    s = ms / 1e3
    achieved = B_PER_ATOM_FRAME * atom_frames / s / 1e9 if s > 0 else 0.0
    return {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_source,
            "launches": launches, "avg_launch_ms": ms / max(1, launches),
            "algorithmic_bytes_per_launch": B_PER_ATOM_FRAME * atom_frames / max(1, launches),
            "bytes_rule": "12 B per (atom, frame) of each timed launch (SURVEY.md 8(d)); achieved = sum(bytes) / "
                          "sum(HIP-event launch time)"}


def rank_roofline(kernel: str, rows, traffic=None, traffic_source=None) -> dict:
    """``roofline`` for every rank's timed launches: ``rows`` = one
    (launches, ms, atom_frames) triple per rank (rank order).  achieved =
    sum(bytes) / sum(launch time) over all ranks; ``per_device_gbs`` each
    rank's own rate, ``slowest_rank_gbs`` / ``slowest_rank`` the minimum."""
    rows = [tuple(float(v) for v in r) for r in rows]
    rf = roofline(kernel, int(sum(r[0] for r in rows)), sum(r[1] for r in rows), sum(r[2] for r in rows),
                  traffic, traffic_source)
    per = [B_PER_ATOM_FRAME * r[2] / (r[1] / 1e3) / 1e9 if r[1] > 0 else None for r in rows]
    live = [(g, i) for i, g in enumerate(per) if g is not None]
    rf["ranks"] = len(rows)
    rf["per_device_gbs"] = per
    rf["per_device_launches"] = [int(r[0]) for r in rows]
    rf["slowest_rank_gbs"], rf["slowest_rank"] = min(live) if live else (None, None)
    rf["slowest_rank_frac"] = rf["slowest_rank_gbs"] / HBM_PEAK_GBS if live else None
    if len(rows) > 1:
        rf["bytes_rule"] += "; summed over every rank's launches (all-reduced before rank 0 prints)"
    return rf


def gather_rank_rows(vals, device=None) -> list:
    """Every rank's ``vals`` (a short list of numbers), in rank order, on
    every rank: each rank fills its row of a zero [world, k] f64 tensor and
    one SUM all-reduce assembles them (works over RCCL and gloo)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [list(vals)]
    w, r = dist.get_world_size(), dist.get_rank()
    t = torch.zeros(w, len(vals), dtype=torch.float64, device=device)
    t[r] = torch.tensor([float(v) for v in vals], dtype=torch.float64)
    dist.all_reduce(t)
    return t.cpu().tolist()


def c1_latency(eng, no_cpu: bool) -> dict:
    """Config C1 shape (BASELINE configs[0]): 3341 atoms, 214 selected, 98
    frames, RMSF.py's two-sweep average alignment -- latency of one full
    RMSF.py computation, HBM-resident (synthetic data of that shape; the adk
    files are not available).  The CPU figure is the numpy restatement of
    the same computation on one core (RMSF.py:23-25 pins one thread/rank)."""
    import numpy as np
    import torch

    from rmsf_amd.pipeline import CapturedPipeline, auto_exact, run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList
    from rmsf_amd.synth import generate, motion_table

    n_atoms, nf = 3341, 98
    sel = np.sort(np.random.default_rng(12).choice(n_atoms, 214, replace=False))
    mt = motion_table(13, nf)
    traj = generate(eng, n_atoms, 0, nf, seed=11, motion=mt)
    src = DeviceSource(traj, sel)
    fl = FrameList(nf)
    for _ in range(5):
        run_pipeline(eng, src, fl, align="average")
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        res = run_pipeline(eng, src, fl, align="average")
    torch.cuda.synchronize()
    gpu_ms = (time.perf_counter() - t0) / reps * 1e3
    cap = CapturedPipeline(eng, src, fl, align="average")
    for _ in range(5):
        cap.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        cap.replay()
    torch.cuda.synchronize()
    graph_ms = (time.perf_counter() - t0) / reps * 1e3
    same = bool(torch.equal(cap.result.rmsf, res.rmsf))
    # the default above is the exact path (aligned, under AUTO_EXACT_FRAMES
    # frames); the frame-parallel path beside it
    for _ in range(5):
        run_pipeline(eng, src, fl, align="average", exact=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fp = run_pipeline(eng, src, fl, align="average", exact=False)
    torch.cuda.synchronize()
    fp_ms = (time.perf_counter() - t0) / reps * 1e3
    out = {"workload": "C1 shape: 3341 atoms, 214 selected, 98 frames, RMSF.py two-sweep",
           "default_path": "exact" if auto_exact("average", nf) else "frame-parallel",
           "gpu_ms_eager": gpu_ms, "gpu_ms_hipgraph": graph_ms, "hipgraph_bitwise_equal": same,
           "gpu_ms_eager_frame_parallel": fp_ms,
           "max_abs_diff_frame_parallel_A": float((fp.rmsf - res.rmsf).abs().max()),
           "sanity": sanity(eng, res.rmsf, nf, seed=11, atoms=sel)}
    if not no_cpu:
        from oracle import rmsf_oracle as O

        host = traj.cpu().numpy()
        t0 = time.perf_counter()
        O.rmsf_script(host, sel, None, size=1, align="average")
        out["cpu_ms_1core_numpy"] = (time.perf_counter() - t0) * 1e3
        out["note"] = "CPU: oracle restatement on 1 core (no XTC decode, no re-selection): optimistic"
    return out


def sanity(eng, rmsf, n_frames: int, seed: int = 0, atoms=None, fatal: bool = True) -> dict:
    """Package-side result check of a timed mode (rmsf_amd.synth.rmsf_sanity:
    every atom's RMSF against the generator's sqrt(3) sigma); a failed check
    ends the bench -- a fast wrong result is not a measurement.  ``fatal``
    False: return the verdict and let the caller end every rank together."""
    from rmsf_amd.synth import rmsf_sanity

    chk = rmsf_sanity(eng, rmsf, n_frames, seed=seed, atoms=atoms)
    if fatal and not chk["ok"]:
        raise SystemExit(f"bench sanity check failed: {chk}")
    return chk


def c4_share_mode(eng, a, headline_avg_ms: float | None, n_atoms: int = 1_000_000, nf: int = 2_500) -> dict:
    """Config C4's per-rank step at N = 8 (BASELINE configs[3]: 1M atoms x
    20k frames over 8 GPUs = 1M x 2,500 per rank), on this one device: the
    one-process form's context step -- rmsf_multi_push_frames with the merge
    shift frame, the sweep recorded for the 2-slab merge, then
    rmsf_multi_chan_merge_root(root=0) streaming it slab by slab (each slab's
    accumulate + fold-pack) -- with the no-op transport (no peers: the
    collective moves nothing; the RMSF is this block's, RMSF.py:65-69)."""
    import torch

    from rmsf_amd.context import PUSH_WELFORD, TRANSPORT_NOOP, Context
    from rmsf_amd.synth import generate

    traj = generate(eng, n_atoms, 0, nf, seed=0)
    torch.cuda.synchronize()
    c = Context(n_atoms, device=eng.device.index)
    try:
        c.set_timing(True)
        Context.multi_set_transport([c], TRANSPORT_NOOP)
        frame0 = traj[0]

        def step():
            Context.multi_push_frames([c], [traj], PUSH_WELFORD, shift_frames=[frame0], merge_slabs=2,
                                      after_torch=False)
            Context.multi_chan_merge([c], root=0)

        for _ in range(max(1, a.mode_warmup)):
            step()
        for w in ("accumulate", "merge"):
            c.kernel_time(w)
        t0 = time.perf_counter()
        for _ in range(a.mode_steps):
            step()
        c.synchronize()
        dt = time.perf_counter() - t0
        k, ms, af = c.kernel_time("accumulate")
        km, mms, _ = c.kernel_time("merge")
        rmsf = c.rmsf()
    finally:
        c.close()
    step_ms = dt / a.mode_steps * 1e3
    peak_ms = B_PER_ATOM_FRAME * n_atoms * nf / (HBM_PEAK_GBS * 1e9) * 1e3
    out = {"workload": f"C4 share: {n_atoms} atoms x {nf} frames (1M x 2,500 = one rank's block of configs[3] at "
                       "N = 8); the one-process context step (2 atom slabs, fold-pack, reduce to root) with a "
                       "no-op transport",
           "atom_frames_per_s": n_atoms * nf * a.mode_steps / dt, "ms_per_step": step_ms,
           "accumulate_launches_per_step": k / a.mode_steps, "accumulate_ms_per_step": ms / a.mode_steps,
           "accumulate_frac": B_PER_ATOM_FRAME * af / (ms / 1e3) / 1e9 / HBM_PEAK_GBS if ms else None,
           "exposed_merge_ms_per_step": mms / max(1, km),
           "floor_peak_ms": peak_ms, "step_over_peak_floor": step_ms / peak_ms,
           "sanity": sanity(eng, rmsf, nf)}
    if headline_avg_ms:
        # the headline stream's measured rate applied to the share's bytes
        # (100k x 2,500 at 0.446 ms scales by 10 to 1M atoms)
        fl = headline_avg_ms * (n_atoms * nf) / (100_000 * 20_000)
        out.update(floor_headline_rate_ms=fl, step_over_headline_rate=step_ms / fl)
    del traj
    torch.cuda.empty_cache()
    return out


def c5_xtc_mode(eng, a, n_atoms: int = 250_000, nf: int = 2048) -> dict:
    """Config C5 (BASELINE configs[4]): a 250k-atom XTC file streamed from the
    host, written untimed from the synthetic generator, then per step read
    (pread into pinned slots), copied to HBM and decompressed on the GPU
    (XtcSource decode="gpu"), the Welford stream consuming each batch --
    read + PCIe + decode inclusive.  The decode kernel's own time is
    measured apart on HBM-resident records (HIP events, torch's stream)."""
    import shutil
    import tempfile

    import numpy as np
    import torch

    from rmsf_amd._lib import call
    from rmsf_amd.pipeline import KernelTimer, run_pipeline
    from rmsf_amd.sources import FrameList, XtcSource
    from rmsf_amd.synth import generate
    from rmsf_amd.xtc import XTCFile, write_xtc

    d = tempfile.mkdtemp(prefix="rmsf_c5_")
    path = os.path.join(d, "c5.xtc")
    try:
        t_w = time.perf_counter()
        for f in range(0, nf, 256):
            n = min(256, nf - f)
            write_xtc(path, generate(eng, n_atoms, f, n, seed=0).cpu().numpy(), append=f > 0)
        t_w = time.perf_counter() - t_w
        src = XtcSource(path, None, decode="gpu", n_threads=16, n_slots=3)
        fl = FrameList(nf)
        run_pipeline(eng, src, fl)
        torch.cuda.synchronize()
        timer = KernelTimer()
        t0 = time.perf_counter()
        for _ in range(a.mode_steps):
            res = run_pipeline(eng, src, fl, timer=timer)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        k, ms, af = timer.totals("accumulate")
        xbytes = os.path.getsize(path)
        # the decode kernel alone: the first 512 frames' records in HBM
        nk = min(512, nf)
        with XTCFile(path) as f:
            rec = [f.record(i) for i in range(nk)]
        o0 = rec[0][0]
        raw = np.fromfile(path, dtype=np.uint32, count=(rec[-1][0] + rec[-1][1] - o0) // 4, offset=o0)
        off = torch.tensor([(o - o0) // 4 for o, _ in rec], dtype=torch.int64, device=eng.device)
        ln = torch.tensor([n // 4 for _, n in rec], dtype=torch.int64, device=eng.device)
        words = torch.as_tensor(raw.view(np.int32)).to(eng.device)
        out = torch.empty((nk, n_atoms, 3), dtype=torch.float32, device=eng.device)
        st = torch.empty(nk, dtype=torch.int32, device=eng.device)
        s = torch.cuda.current_stream(eng.device)

        def dec():
            call("rmsf_xtc_decode_records", words.data_ptr(), off.data_ptr(), ln.data_ptr(), nk, n_atoms,
                 out.data_ptr(), 3 * n_atoms, st.data_ptr(), s.cuda_stream)

        dec()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for e0, e1 in evs:
            e0.record(s)
            dec()
            e1.record(s)
        torch.cuda.synchronize()
        dec_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
        ok_status = bool((st == 0).all())
        chk = sanity(eng, res.rmsf, nf)
        del src, words, out
        torch.cuda.empty_cache()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"workload": "C5: 250k-atom XTC (precision 1000, written untimed from the generator) streamed from the "
                        "host: pread into pinned slots, H2D of the compressed records, GPU decode, Welford stream",
            "n_atoms": n_atoms, "n_frames": nf, "frames_per_s": nf * a.mode_steps / dt,
            "atom_frames_per_s": n_atoms * nf * a.mode_steps / dt, "ms_per_step": dt / a.mode_steps * 1e3,
            "xtc_bytes": xbytes, "h2d_gbs": xbytes * a.mode_steps / dt / 1e9, "host_link_spec_gbs": 63.0,
            "h2d_over_link": xbytes * a.mode_steps / dt / 1e9 / 63.0,
            "decoded_frame_gbs": B_PER_ATOM_FRAME * n_atoms * nf * a.mode_steps / dt / 1e9,
            "decode_kernel": {"frames": nk, "avg_ms": dec_ms, "frames_per_s": nk / (dec_ms / 1e3),
                              "decoded_gbs": B_PER_ATOM_FRAME * n_atoms * nk / (dec_ms / 1e3) / 1e9,
                              "all_frames_ok": ok_status},
            "accumulate_avg_ms": ms / max(1, k), "xtc_write_s_untimed": t_w, "sanity": chk}


# HBM bytes per step of the sparse modes, from the L2's read requests by size
# and WRITE_SIZE (rocprofv3 --pmc passes of tools/sparse_once.py, round 6;
# profiles/r06_workloads/pmc_sparse_c4.txt) -- a committed measurement, like
# the headline's traffic, not a counter of this run
SPARSE_PMC = {
    "c3_ca_like": {"regathered_read_gb": 48.14, "compacted_read_gb": 26.63, "compacted_written_gb": 2.43},
    "average_ca_like": {"regathered_read_gb": 96.24, "compacted_read_gb": 31.80, "compacted_written_gb": 2.43},
}


def sparse_selection_modes(eng, a, traj, n_atoms: int, n_total: int) -> dict:
    """RMSF.py's real workload shape: a sparse selection of the system
    (``select_atoms("protein and name CA")``, RMSF.py:77,126 -- 214 of 47,681
    atoms) on the headline trajectory (100k atoms x 20k frames, aligned
    motion), HBM-resident.  Every 10th atom (CA-like) under
    C3's frame-0 alignment and RMSF.py's two sweeps, and the adk density (1 in
    220) under the two sweeps -- each timed with the selected rows compacted
    by the first pass (the default below the compaction densities) and re-gathered
    by every pass (compact=False), same bits.  Rates and roofline fractions
    count the SELECTED bytes (12 B per selected atom-frame per sweep); the
    gather reads every 128-B line that holds a selected atom, which at 1 in
    10 is nearly every line of the frames."""
    import numpy as np
    import torch

    from rmsf_amd.pipeline import KernelTimer, run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList

    fl = FrameList(n_total)
    out = {}
    for name, stride, align in (("c3_ca_like", 10, "frame0"), ("average_ca_like", 10, "average"),
                                ("average_adk_density", 220, "average")):
        sel = np.arange(0, n_atoms, stride)
        src = DeviceSource(traj, sel, n_traj=n_total)
        n_sel = len(sel)
        sweeps = 2 if align == "average" else 1
        row = {"selection": f"every {stride}th atom: {n_sel} of {n_atoms}", "align": align, "sweeps": sweeps}
        res = {}
        for compact in (True, False):
            def run(timer=None):
                return run_pipeline(eng, src, fl, align=align, timer=timer, compact=compact)

            for _ in range(max(1, a.mode_warmup)):
                run()
            torch.cuda.synchronize()
            t = KernelTimer()
            t0 = time.perf_counter()
            for _ in range(a.mode_steps):
                r = run(t)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[compact] = r.rmsf
            ks, s_ms, _ = t.totals("superpose")
            ka, a_ms, _ = t.totals("accumulate")
            step_ms = dt / a.mode_steps * 1e3
            sel_bytes = B_PER_ATOM_FRAME * n_sel * n_total * sweeps
            key = "compacted" if compact else "regathered"
            row[key] = {"ms_per_step": step_ms, "atom_frames_per_s": n_sel * n_total * a.mode_steps / dt,
                        "selected_gbs": sel_bytes / (step_ms / 1e3) / 1e9,
                        "frac_of_single_read_roofline": sel_bytes / (step_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                        "superpose_ms_per_step": s_ms / a.mode_steps, "superpose_launches": ks // a.mode_steps,
                        "accumulate_ms_per_step": a_ms / a.mode_steps, "accumulate_launches": ka // a.mode_steps}
        row["speedup_compacted"] = row["regathered"]["ms_per_step"] / row["compacted"]["ms_per_step"]
        if name in SPARSE_PMC:  # bytes moved per selected byte, regathered vs compacted
            pm = dict(SPARSE_PMC[name])
            sel_gb = B_PER_ATOM_FRAME * n_sel * n_total * sweeps / 1e9
            pm["selected_gb"] = sel_gb
            pm["regathered_over_selected"] = pm["regathered_read_gb"] / sel_gb
            pm["compacted_over_selected"] = (pm["compacted_read_gb"] + pm["compacted_written_gb"]) / sel_gb
            pm["source"] = "profiles/r06_workloads/pmc_sparse_c4.txt"
            row["traffic_pmc"] = pm
        row["same_bits"] = bool(torch.equal(res[True], res[False]))
        if not row["same_bits"]:
            raise SystemExit(f"bench: compacted and re-gathered results differ ({name})")
        # reported, not fatal: fitting on 1 atom in 220 leaves a rotation error
        # of ~1e-3 rad (sigma / (R sqrt(n_sel))) that adds up to ~0.1 A at the
        # box corners, beyond the 5 % rule for the quietest atoms
        row["sanity"] = sanity(eng, res[True], n_total, atoms=sel, fatal=False)
        out[name] = row
        del src, res
        torch.cuda.empty_cache()
    return out


def cpu_baselines(a, wl) -> tuple[dict | None, dict | None]:
    """Before any GPU call: RMSF.py's two sweeps (the north star's ``mpirun -n
    <cores> python RMSF.py``) and the unaligned C2 sweep, both on the usable
    host cores, bounded samples of the same 100k-atom trajectory."""
    from oracle import cpu_baseline
    from rmsf_amd.synth import motion_table  # numpy only: no GPU touched

    cores = cpu_baseline.available_cores()[0]
    n = wl["n_atoms"]
    avg = cpu_baseline.run(n, a.cpu_average_frames, align="average",
                           motion=motion_table(1, a.cpu_average_frames * cores))
    flat = cpu_baseline.run(n, a.cpu_frames, align="none")
    return avg, flat


def base_line(a, wl, n_gpus: int, dt: float, parallelism: str) -> dict:
    n_atoms, n_total = wl["n_atoms"], wl["n_total"]
    return {
        "metric": METRIC,
        "value": n_total * n_atoms * a.steps / dt,
        "unit": "atom-frames/s",
        "n_gpus": n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: counter-based generator, fp32 frames resident in HBM (generated on device)",
        "config": {"workload": wl["name"], "n_atoms": n_atoms, "n_frames_total": n_total,
                   "n_frames_per_gpu": n_total // n_gpus,
                   "selection": "all atoms", "align": wl["align"], "parallelism": parallelism},
    }


# ---------------------------------------------------------------------------
# one process, N devices (no launcher): the C ABI's contexts


def main_single_process(a, wl, cpu) -> None:
    """``--gpus N`` with no WORLD_SIZE: one context per device, each device's
    RMSF.py:65-69 block generated in its HBM; every step pushes all blocks at
    once (rmsf_multi_push_frames: one host thread per device, no host
    synchronisation), then the contexts' merge -- the torchrun rank step's
    shape: one collective of moments about frame 0 (unaligned) or the
    reference (aligned), a reduce to context 0 with ``--merge root``
    (RMSF.py:143), atom slabs from 1M atoms.  Exchanges over ncclCommInitAll
    communicators; a --rehearse device list uses the in-process host fold, or
    a no-op transport for host-cost timing."""
    import torch

    from rmsf_amd import parallel
    from rmsf_amd.context import (PUSH_ALIGN_SUM, PUSH_ALIGN_WELFORD, PUSH_WELFORD, TRANSPORT_NOOP, Context)
    from rmsf_amd.engine import Engine
    from rmsf_amd.synth import generate, motion_table

    if wl.get("host"):
        raise SystemExit("one-process multi-GPU runs cover the HBM-resident workloads (c2, c3, average, c4)")
    devs, rehearsal = device_plan(a.gpus, torch.cuda.device_count(), a.rehearse)
    n = len(devs)
    n_atoms, n_total, align = wl["n_atoms"], wl["n_total"], wl["align"]
    blocks = parallel.blocks(n_total, n)
    motion = motion_table(1, n_total) if align else None
    ctxs, trajs, frame0 = [], [], []
    for d, (b0, b1) in zip(devs, blocks):
        with torch.cuda.device(d):
            eng = Engine(torch.device("cuda", d))
            trajs.append(generate(eng, n_atoms, b0, b1 - b0, seed=0, motion=motion))
            # every rank reads frame 0 itself (RMSF.py:80-87): an input, like
            # the block -- the reference (aligned) or the merge's shift
            frame0.append(generate(eng, n_atoms, 0, 1, seed=0, motion=motion)[0])
            torch.cuda.synchronize(d)
        c = Context(n_atoms, device=d)
        c.set_timing(True)
        ctxs.append(c)
    if not rehearsal:
        Context.init_all(ctxs)  # ncclCommInitAll, also for one device (--one-process): the RCCL merge path
    noop = rehearsal and a.rehearse_transport == "noop"
    if noop:
        Context.multi_set_transport(ctxs, TRANSPORT_NOOP)
    root = 0 if (a.merge == "root" and n > 1) else None
    slabs = 0 if a.merge_slabs is None else max(1, a.merge_slabs)   # C ABI: 0 = auto, 1 = off
    kw = dict(after_torch=False)  # the blocks were generated and synchronised above

    def step():
        if align == "average":
            Context.multi_push_frames(ctxs, trajs, PUSH_ALIGN_SUM, ref_frames=frame0, **kw)   # RMSF.py:80-105
            Context.multi_allreduce_sum(ctxs)                                                 # RMSF.py:107-110
            for c in ctxs:
                c.set_reference_average()                                                     # RMSF.py:111-118
            Context.multi_push_frames(ctxs, trajs, PUSH_ALIGN_WELFORD, **kw)                  # RMSF.py:120-138
        elif align == "frame0":
            Context.multi_push_frames(ctxs, trajs, PUSH_ALIGN_WELFORD, ref_frames=frame0, **kw)
        else:
            Context.multi_push_frames(ctxs, trajs, PUSH_WELFORD, shift_frames=frame0 if n > 1 else None,
                                      merge_slabs=slabs, **kw)
        Context.multi_chan_merge(ctxs, root=root)                                             # RMSF.py:140-143
        # RMSF.py:145-146: finalised in the merge (n > 1) / by rmsf() below

    for _ in range(a.warmup):
        step()
    for c in ctxs:  # drop the warm-up's launch records (synchronises)
        c.kernel_time("accumulate"), c.kernel_time("superpose"), c.kernel_time("merge")
        c.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step()
        host_s += time.perf_counter() - h0
    for c in ctxs:
        c.synchronize()
    dt = time.perf_counter() - t0
    acc = [c.kernel_time("accumulate") for c in ctxs]
    sup = [c.kernel_time("superpose") for c in ctxs]
    mer = [c.kernel_time("merge") for c in ctxs]
    rmsf = ctxs[root or 0].rmsf()
    transport = ("REHEARSAL: device 0 listed %d times, %s" % (n, "no-op exchanges (host-cost timing; the merged "
                 "result is not global)" if noop else "in-process host fold") if rehearsal
                 else "RCCL via ncclCommInitAll")
    par = f"one process, {n} device contexts (RMSF.py:65-69 blocks), {transport}, exact k-way Chan merge"
    out = base_line(a, wl, n, dt, par)
    out["devices"] = devs
    out["rehearsal"] = rehearsal
    out["host_enqueue_ms_per_step"] = host_s / a.steps * 1e3
    if n > 1:
        out["config"]["merge"] = ("reduce to context 0 (RMSF.py:143)" if root == 0 else "all-reduce") + \
            " of moments about a common shift (one collective)"
    kname = ("k_accum_split_sk" if align else "k_welford_flat_sk")
    out["roofline"] = rank_roofline(kname, acc)
    if align:
        ms, af = sum(x[1] for x in sup), sum(x[2] for x in sup)
        out["superpose"] = {"launches": sum(x[0] for x in sup), "avg_launch_ms": ms / max(1, sum(x[0] for x in sup)),
                            "gflops": FLOP_PER_ATOM_FRAME_SUPERPOSE * af / (ms / 1e3) / 1e9 if ms else None}
    if n > 1:
        # each context's merge as its stream saw it: HIP events from its packed
        # moments to its finished result (the collective, the wait for the
        # slowest context, the unpack; with slabs the part after the last slab)
        per = [m[1] / max(1, m[0]) for m in mer]
        out["merge_timing"] = {"per_device_ms_per_step": per, "max_ms_per_step": max(per),
                               "rule": "HIP events on each context's stream around its part of "
                                       "rmsf_multi_chan_merge_root, per timed step (rmsf_ctx_kernel_time MERGE)"}
    out["cpu_baseline"] = cpu
    out["rmsf_checksum"] = float(rmsf.sum())
    if not noop:
        with torch.cuda.device(devs[root or 0]):
            out["sanity"] = sanity(Engine(torch.device("cuda", devs[root or 0])), rmsf, n_total)
    print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()


# ---------------------------------------------------------------------------
# one process per GPU (torch.distributed) or N=1


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    launched = "WORLD_SIZE" in os.environ
    if launched and a.gpus != world and not a.backend == "gloo":
        raise SystemExit(f"--gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    single_multi = not launched and (a.gpus > 1 or a.one_process)
    n_gpus = a.gpus if single_multi else world
    wl = resolve(a, n_gpus)
    n_atoms, n_total = wl["n_atoms"], wl["n_total"]

    # -- CPU baseline first: no process has touched the GPU yet ---------------
    cpu_avg = cpu_flat = None
    if rank == 0 and n_gpus == 1 and not a.no_cpu_baseline and not wl.get("host"):
        cpu_avg, cpu_flat = cpu_baselines(a, wl)
    cpu = None
    if cpu_avg is not None:
        cpu = dict(cpu_avg)
        cpu["unaligned"] = cpu_flat  # the headline workload's own sweep (C2), second figure

    if single_multi:
        main_single_process(a, wl, cpu)
        return

    import torch
    import torch.distributed as dist

    if a.backend == "gloo":  # rehearsal: all ranks share the visible device(s)
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.backend)
    from rmsf_amd import parallel
    from rmsf_amd.engine import Engine
    from rmsf_amd.pipeline import KernelTimer, run_pipeline
    from rmsf_amd.sources import DeviceSource, FrameList
    from rmsf_amd.synth import generate, motion_table

    eng = Engine(torch.device("cuda", local))
    if world > 1:
        # RCCL sets its connections up at the first collective: do that once,
        # untimed, at the merge's message size, so it is not charged to a step
        # even when --warmup 0
        _t = torch.zeros(3 * n_atoms, dtype=torch.float64, device=eng.device)
        dist.all_reduce(_t)
        if a.merge == "root":
            dist.reduce(_t, dst=0)
        if a.merge == "scatter":
            _per = -(-n_atoms // world)
            _o = torch.zeros(6 * _per, dtype=torch.float64, device=eng.device)
            parallel_rs = torch.zeros(6 * _per * world, dtype=torch.float64, device=eng.device)
            from rmsf_amd import parallel as _p
            _p.reduce_scatter_sum_(_o, parallel_rs)
            _p.gather_(_o[:_per], 0)
            del _o, parallel_rs
        dist.barrier()
        torch.cuda.synchronize()
        del _t
    b0, b1 = parallel.blocks(n_total, world)[rank]
    n_local = b1 - b0
    motion = motion_table(1, n_total) if wl["align"] else None
    traj = generate(eng, n_atoms, b0, n_local, seed=0, motion=motion)
    torch.cuda.synchronize()
    h2d_bytes = None
    if wl.get("host"):
        # C5: the frames live in (pageable) host memory and every step streams
        # them through the stager: host gather -> pinned slot -> H2D -> kernels
        from rmsf_amd.sources import HostSource

        host = traj.cpu().numpy()
        del traj
        torch.cuda.empty_cache()
        if wl.get("xtc"):
            import tempfile

            from rmsf_amd.sources import XtcSource
            from rmsf_amd.xtc import write_xtc

            if world > 1:
                raise SystemExit("c5xtc is a single-GPU I/O workload")
            xtc_dir = tempfile.mkdtemp(prefix="rmsf_c5_")
            xtc_path = os.path.join(xtc_dir, "c5.xtc")
            t_w = time.perf_counter()
            for f in range(0, n_local, 256):  # untimed: produce the input file
                write_xtc(xtc_path, host[f:f + 256], append=f > 0)
            t_w = time.perf_counter() - t_w
            del host
            src = XtcSource(xtc_path, None, batch_frames=a.stager_batch, decode=a.xtc_decode,
                            n_threads=a.stager_threads if a.xtc_decode == "host" else max(a.stager_threads, 16),
                            n_slots=3, cache=a.xtc_cache)
        else:
            if a.host_layout == "soa":  # untimed: the same frames as coordinate planes
                import numpy as np

                host = np.ascontiguousarray(host.transpose(0, 2, 1))
            src = HostSource(host, None, batch_frames=a.stager_batch, n_threads=a.stager_threads, offset=b0,
                             n_traj=n_total, cache=a.host_cache, layout=a.host_layout)
    else:
        src = DeviceSource(traj, offset=b0, n_traj=n_total)
    fl = FrameList(n_total)

    def run(align, timer=None):
        if hasattr(src, "drop_cache"):
            src.drop_cache()  # every step streams the file again
        return run_pipeline(eng, src, fl, align=align, block=(b0, b1), ref_owner=0, n_splits=a.splits,
                            max_batch=a.batch_frames, timer=timer, merge_slabs=a.merge_slabs,
                            merge_root=0 if a.merge in ("root", "scatter") else None,
                            merge_scatter=a.merge == "scatter")

    def timed(align, steps, warmup):
        timer = KernelTimer()
        for _ in range(warmup):
            run(align)
        torch.cuda.synchronize()
        parallel.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = run(align, timer)
        torch.cuda.synchronize()
        parallel.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=eng.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt, timer, res

    dt, timer, res = timed(wl["align"], a.steps, a.warmup)
    transport = "RCCL" if a.backend == "nccl" else f"{a.backend} (REHEARSAL: ranks may share a device)"
    par = (f"frame-sharded x{world} (RMSF.py:65-69 blocks), one process per GPU, {transport} Chan merge"
           if world > 1 else "1 GPU")
    out = base_line(a, wl, world, dt, par)
    if world > 1:
        out["config"]["merge_slabs"] = res.extras.get("merge_slabs", 0)
        out["config"]["merge"] = {"root": "reduce to rank 0 (RMSF.py:143)", "all": "all-reduce",
                                  "scatter": "reduce-scatter by atom slices, each rank finishes its slice, RMSF "
                                             "gathered to rank 0 (RMSF.py:143's result)"}[a.merge]
    launches, acc_ms, acc_af = timer.totals("accumulate")
    traffic = load_traffic(a.workload, n_atoms, n_local) if launches == a.steps else None
    kname = (("k_accum_atoms" if wl["align"] else "k_welford_flat") if a.splits
             else ("k_accum_split_sk" if wl["align"] else "k_welford_flat_sk"))
    # every rank's launches (one all-reduce, after the timed region)
    coll_dev = eng.device if a.backend == "nccl" else None
    rows = gather_rank_rows([launches, acc_ms, acc_af], coll_dev)
    out["roofline"] = rank_roofline(kname, rows, traffic, f"profiles/pmc_{a.workload}.json" if traffic else None)
    if world > 1:
        # the cross-rank merge as each rank's launching stream saw it: HIP events
        # around the collective + unpack/finalise (waits for the slowest rank
        # included; with atom slabs, only the exposed part after the last slab)
        mrows = gather_rank_rows(list(timer.totals("merge")), coll_dev)
        out["merge_timing"] = {"per_rank_ms_per_step": [r[1] / max(1.0, r[0]) for r in mrows],
                               "max_ms_per_step": max(r[1] / max(1.0, r[0]) for r in mrows),
                               "rule": "HIP events on the launching stream around the merge collective and the "
                                       "unpack/finalise, per timed step"}
    out["cpu_baseline"] = cpu
    # the merged result (on rank 0 only with the default reduce-to-root merge)
    out["rmsf_checksum"] = float(res.rmsf.sum()) if res.rmsf is not None else None
    if res.rmsf is not None:
        out["sanity"] = sanity(eng, res.rmsf, n_total, fatal=False)
    # the verdict is collective: only the merge's root holds the RMSF, and a
    # rank that left alone would leave the others waiting in the collectives
    # below -- every rank ends together on a failed check
    if any(r[0] for r in gather_rank_rows([0.0 if out.get("sanity", {"ok": True})["ok"] else 1.0], coll_dev)):
        raise SystemExit(f"bench sanity check failed: {out.get('sanity', 'on the merge root')}")
    # whole-step rate in algorithmic bytes (incl. merges, finalise, launch gaps)
    out["pipeline_hbm_gbs"] = B_PER_ATOM_FRAME * n_atoms * n_local * a.steps / dt / 1e9
    if wl["align"]:
        srows = gather_rank_rows(list(timer.totals("superpose")), coll_dev)
        k, s_ms, s_af = (sum(r[i] for r in srows) for i in range(3))
        if k:
            out["superpose"] = {"launches": int(k), "avg_launch_ms": s_ms / k,
                                "gflops": FLOP_PER_ATOM_FRAME_SUPERPOSE * s_af / (s_ms / 1e3) / 1e9,
                                "fp64_peak_tflops_spec": FP64_PEAK_TFS,
                                "hbm_gbs": B_PER_ATOM_FRAME * s_af / (s_ms / 1e3) / 1e9,
                                "per_device_hbm_gbs": [B_PER_ATOM_FRAME * r[2] / (r[1] / 1e3) / 1e9 if r[1] else None
                                                       for r in srows]}

    if wl.get("host"):
        # bytes that actually cross PCIe per step: the staged selection rows of
        # a host array, or the compressed XTC records (GPU decode) / decoded
        # selection rows (host decode)
        sweeps = 2 if wl["align"] == "average" and not (a.host_cache or a.xtc_cache) else 1
        decoded = B_PER_ATOM_FRAME * n_atoms * n_local
        if wl.get("xtc") and a.xtc_decode == "gpu":
            h2d_bytes = os.path.getsize(xtc_path) * sweeps
        else:
            h2d_bytes = decoded * sweeps
        out["stager"] = {"h2d_bytes_per_step": h2d_bytes,
                         "h2d_gbs": h2d_bytes * a.steps / dt / 1e9,
                         "decoded_frame_gbs": decoded * a.steps / dt / 1e9,
                         "host_cache": bool(getattr(src, "cache", None) is not None),
                         "host_layout": getattr(src, "layout", "fac"),
                         "threads": a.stager_threads, "batch_frames": src.batch_frames,
                         "host_link_spec_gbs": 63.0}
        if wl.get("xtc"):
            out["stager"].update(xtc_decode=a.xtc_decode, xtc_cache=a.xtc_cache,
                                 xtc_bytes=os.path.getsize(xtc_path), xtc_write_s=t_w,
                                 xtc_frames_per_s=n_local * a.steps / dt)
        out["data"] = "synthetic frames in host memory" + (" written to an XTC file" if wl.get("xtc") else "")
        out["roofline"]["note"] = "C5 is PCIe/host bound; the kernel roofline above is the device-side launches"

    # -- aligned modes at N=1 (reported beside the headline) ------------------
    if world == 1 and not a.no_modes and wl["align"] is None and not wl.get("host"):
        # exact=True on the headline's frames: RMSF.py:137-138 as written
        # (k_welford_seq), bit-identical to the reference recurrence
        def run_exact(timer=None):
            return run_pipeline(eng, src, fl, block=(b0, b1), max_batch=a.batch_frames, timer=timer, exact=True)

        for _ in range(max(1, a.mode_warmup)):
            run_exact()
        torch.cuda.synchronize()
        xt = KernelTimer()
        t0 = time.perf_counter()
        for _ in range(a.mode_steps):
            res_x = run_exact(xt)
        torch.cuda.synchronize()
        xdt = time.perf_counter() - t0
        k_x, x_ms, x_af = xt.totals("accumulate")
        exact_mode = {
            "atom_frames_per_s": n_total * n_atoms * a.mode_steps / xdt,
            "ms_per_step": xdt / a.mode_steps * 1e3,
            "kernel": "k_welford_seq",
            "avg_launch_ms": x_ms / max(1, k_x),
            "hbm_frac": B_PER_ATOM_FRAME * x_af / (x_ms / 1e3) / 1e9 / HBM_PEAK_GBS if x_ms > 0 else None,
            "max_abs_rmsf_diff_vs_headline": float((res_x.rmsf - res.rmsf).abs().max()),
            "sanity": sanity(eng, res_x.rmsf, n_total),
            "note": "RMSF.py:120-146 with the reference's own arithmetic, bit for bit (tests/test_gpu_exact.py, "
                    "tests/test_reduce_order.py)"}
        del traj, src
        torch.cuda.empty_cache()
        motion = motion_table(1, n_total)
        traj = generate(eng, n_atoms, b0, n_local, seed=0, motion=motion)
        torch.cuda.synchronize()
        src = DeviceSource(traj, offset=b0, n_traj=n_total)
        modes = {"c2_exact": exact_mode}
        for name, align in (("c3_frame0", "frame0"), ("rmsf_py_average", "average")):
            mdt, mt, mres = timed(align, a.mode_steps, max(1, a.mode_warmup))
            sweeps = 2 if align == "average" else 1
            af = n_total * n_atoms * a.mode_steps / mdt
            k_s, s_ms, s_af = mt.totals("superpose")
            k_a, a_ms, a_af = mt.totals("accumulate")
            modes[name] = {
                "atom_frames_per_s": af,
                "ms_per_step": mdt / a.mode_steps * 1e3,
                "sweeps": sweeps,
                "hbm_gbs_algorithmic": af * B_PER_ATOM_FRAME * sweeps / 1e9,
                "superpose_avg_ms": s_ms / max(1, k_s),
                "superpose_gflops": FLOP_PER_ATOM_FRAME_SUPERPOSE * s_af / (s_ms / 1e3) / 1e9,
                "superpose_hbm_gbs": B_PER_ATOM_FRAME * s_af / (s_ms / 1e3) / 1e9,
                "accumulate_avg_ms": a_ms / max(1, k_a),
                "accumulate_hbm_gbs": B_PER_ATOM_FRAME * a_af / (a_ms / 1e3) / 1e9,
                "sanity": sanity(eng, mres.rmsf, n_total),
            }
            # the aligned design reads each frame twice per sweep (DESIGN §4,
            # "Why the aligned path reads each frame twice"); against a
            # roofline of ONE read per sweep (12 B per atom-frame per sweep)
            # the whole computation runs at:
            modes[name]["frac_of_single_read_roofline"] = af * B_PER_ATOM_FRAME * sweeps / 1e9 / HBM_PEAK_GBS
        if cpu is not None:
            modes["rmsf_py_average"]["cpu_baseline"] = {
                "value": cpu["value"], "cores": cpu["cores"], "sample": cpu["sample"],
                "gpu_over_cpu": modes["rmsf_py_average"]["atom_frames_per_s"] / cpu["value"]}
        modes.update(sparse_selection_modes(eng, a, traj, n_atoms, n_total))
        modes["c1_rmsf_py"] = c1_latency(eng, a.no_cpu_baseline)
        del traj, src
        torch.cuda.empty_cache()
        if not a.no_io_modes:
            modes["c4_share"] = c4_share_mode(eng, a, out["roofline"]["avg_launch_ms"])
            modes["c5_xtc"] = c5_xtc_mode(eng, a)
        out["modes"] = modes
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
