#!/usr/bin/env python3
"""Headline benchmark: atom-frames/s of the frame-parallel RMSF path on MI355X.

  python bench.py [--gpus N --steps K --warmup W]            (N=1)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

One "step" = one full RMSF pass of the hot path over the rank's frame block
(the per-frame Welford accumulator over every frame, the in-GPU Chan merge of
the frame tiles, the cross-GPU Chan merge over RCCL, the finalise), with the
synthetic trajectory already resident in HBM.  Workload per GPU (weak
scaling, frame-sharded by the RMSF.py:65-69 blocks):
  c2 (default): 100k atoms x 20k frames fp32 per GPU, no alignment
                (BASELINE.json configs[1]); N GPUs hold 20k*N frames.
  c4:           1M atoms x 2.5k frames per GPU (at N=8 = configs[3], 240 GB).
At N=1 the aligned configurations are measured too and reported under
"modes" (C3 = QCP alignment to frame 0; RMSF.py's own two-sweep "average").

Rank 0 prints ONE JSON line.  ``roofline`` is measured live with HIP events
around the dominant kernel (k_welford_flat_sk, the balanced-grid Welford
stream; k_welford_flat with --splits) on its launch stream;
``cpu_baseline`` is the oracle's numpy restatement of RMSF.py's per-rank loop
timed on this host's cores (run before the GPU is touched).
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

WORKLOADS = {
    "c2": dict(n_atoms=100_000, frames_per_gpu=20_000, align=None,
               name="C2: synthetic 100k atoms x 20k frames fp32 per GPU, no alignment, fp64 Welford"),
    "c3": dict(n_atoms=100_000, frames_per_gpu=20_000, align="frame0",
               name="C3: synthetic 100k atoms x 20k frames fp32 per GPU, QCP alignment to frame 0"),
    "average": dict(n_atoms=100_000, frames_per_gpu=20_000, align="average",
                    name="RMSF.py two-sweep: 100k atoms x 20k frames per GPU, align to frame 0, average, re-align"),
    "c4": dict(n_atoms=1_000_000, frames_per_gpu=2_500, align=None,
               name="C4 share: synthetic 1M atoms x 2.5k frames fp32 per GPU (N=8: 1M x 20k, 240 GB)"),
    "c5": dict(n_atoms=250_000, frames_per_gpu=1_000, align=None, host=True,
               name="C5 (pre-decoded): 250k atoms x 1k frames fp32 in host memory, streamed via the pinned "
                    "multi-buffer stager (PCIe-inclusive rate; no XTC decode)"),
    "c5xtc": dict(n_atoms=250_000, frames_per_gpu=2048, align=None, host=True, xtc=True,
                  name="C5: 250k-atom XTC file (precision 1000) streamed from the host and decoded "
                       "(--xtc-decode gpu: compressed records via pinned slots, decompressed on the GPU; host: "
                       "decoded on host threads into the pinned stager); read + PCIe + decode inclusive"),
}


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--n-atoms", type=int, default=None)
    ap.add_argument("--frames-per-gpu", type=int, default=None)
    ap.add_argument("--splits", type=int, default=None)
    ap.add_argument("--batch-frames", type=int, default=None, help="aligned modes: frames per superpose batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=640, help="frames per CPU process in the baseline sample")
    ap.add_argument("--no-modes", action="store_true", help="skip the aligned-mode measurements at N=1")
    ap.add_argument("--mode-steps", type=int, default=3)
    ap.add_argument("--stager-threads", type=int, default=4)
    ap.add_argument("--stager-batch", type=int, default=None, help="c5: frames per staged batch")
    ap.add_argument("--xtc-decode", choices=["gpu", "host"], default="gpu",
                    help="c5xtc: decompress the XTC records on the GPU (default) or on host threads")
    ap.add_argument("--xtc-cache", action="store_true",
                    help="c5xtc (GPU decode): keep decoded frames in HBM within a step (RMSF.py's second sweep "
                         "reads them from HBM); dropped before every step, so each step decodes once")
    ap.add_argument("--host-cache", action="store_true",
                    help="c5: keep the staged frames in HBM within a step (RMSF.py's second sweep reads them there)")
    ap.add_argument("--align", choices=["none", "frame0", "average"], default=None, help="override the workload's")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL; gloo only "
                                                     "to rehearse several ranks on one GPU)")
    return ap.parse_args()


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


def c1_latency(eng, no_cpu: bool) -> dict:
    """Config C1 shape (BASELINE configs[0]): 3341 atoms, 214 selected, 98
    frames, RMSF.py's two-sweep average alignment -- latency of one full
    RMSF.py computation, HBM-resident (synthetic data of that shape; the adk
    files are not available).  The CPU figure is the numpy restatement of
    the same computation on one core (RMSF.py:23-25 pins one thread/rank)."""
    import numpy as np
    import torch

    from rmsf_amd.pipeline import run_pipeline
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
    from rmsf_amd.pipeline import CapturedPipeline

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
    out = {"workload": "C1 shape: 3341 atoms, 214 selected, 98 frames, RMSF.py two-sweep",
           "gpu_ms_eager": gpu_ms, "gpu_ms_hipgraph": graph_ms, "hipgraph_bitwise_equal": same}
    if not no_cpu:
        from oracle import rmsf_oracle as O

        host = traj.cpu().numpy()
        t0 = time.perf_counter()
        O.rmsf_script(host, sel, None, size=1, align="average")
        out["cpu_ms_1core_numpy"] = (time.perf_counter() - t0) * 1e3
        out["note"] = "CPU: oracle restatement on 1 core (no XTC decode, no re-selection): optimistic"
    return out


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    wl = dict(WORKLOADS[a.workload])
    if a.n_atoms:
        wl["n_atoms"] = a.n_atoms
    if a.frames_per_gpu:
        wl["frames_per_gpu"] = a.frames_per_gpu
    if a.align is not None:
        wl["align"] = None if a.align == "none" else a.align
    n_atoms, per_gpu = wl["n_atoms"], wl["frames_per_gpu"]

    # -- CPU baseline first: no process has touched the GPU yet ---------------
    cpu = cpu_c3 = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle import cpu_baseline
        cpu = cpu_baseline.run(n_atoms, a.cpu_frames, align="none")
        if not a.no_modes and wl["align"] is None and not wl.get("host"):
            from rmsf_amd.synth import motion_table as _mt  # numpy only: no GPU touched
            cpu_c3 = cpu_baseline.run(n_atoms, max(1, a.cpu_frames // 4), align="frame0",
                                      motion=_mt(1, per_gpu))

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
        dist.barrier()
        torch.cuda.synchronize()
        del _t
    n_total = per_gpu * world
    b0, b1 = parallel.blocks(n_total, world)[rank]
    n_local = b1 - b0
    motion = motion_table(1, n_total) if wl["align"] else None
    traj = generate(eng, n_atoms, b0, n_local, seed=0, motion=motion)
    torch.cuda.synchronize()
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
            src = HostSource(host, None, batch_frames=a.stager_batch, n_threads=a.stager_threads, offset=b0,
                             n_traj=n_total, cache=a.host_cache)
    else:
        src = DeviceSource(traj, offset=b0, n_traj=n_total)
    fl = FrameList(n_total)

    def run(align, timer=None):
        if hasattr(src, "drop_cache"):
            src.drop_cache()  # every step streams the file again
        return run_pipeline(eng, src, fl, align=align, block=(b0, b1), ref_owner=0, n_splits=a.splits,
                            max_batch=a.batch_frames, timer=timer)

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
    value = n_total * n_atoms * a.steps / dt
    acc_ms = timer.ms("accumulate")
    kern_s = sum(acc_ms) / len(acc_ms) / 1e3
    bytes_launch = B_PER_ATOM_FRAME * n_atoms * n_local
    achieved = bytes_launch / kern_s / 1e9
    traffic = load_traffic(a.workload, n_atoms, n_local)
    out = {
        "metric": "atom-frames/sec (RMSF) + achieved HBM GB/s fraction",
        "value": value,
        "unit": "atom-frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": dt / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: counter-based generator, fp32 frames resident in HBM (generated on device)",
        "config": {"workload": wl["name"], "n_atoms": n_atoms, "n_frames_per_gpu": per_gpu,
                   "n_frames_total": n_total, "selection": "all atoms", "align": wl["align"],
                   "parallelism": f"frame-sharded x{world} (RMSF.py:65-69 blocks), RCCL Chan merge"},
        "roofline": {"bound": "hbm", "kernel": ("k_accum_atoms" if wl["align"] else "k_welford_flat")
                     + ("" if a.splits else "_sk"),
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": f"profiles/pmc_{a.workload}.json" if traffic else None,
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "avg_launch_ms": kern_s * 1e3, "launches": len(acc_ms)},
        "cpu_baseline": cpu,
        # whole-step rate in algorithmic bytes (incl. merges, finalise, launch gaps)
        "pipeline_hbm_gbs": B_PER_ATOM_FRAME * n_atoms * n_local * a.steps / dt / 1e9,
    }
    if wl["align"]:
        sup_ms = timer.ms("superpose")
        if sup_ms:
            s = sum(sup_ms) / len(sup_ms) / 1e3
            out["superpose"] = {"avg_launch_ms": s * 1e3,
                                "gflops": FLOP_PER_ATOM_FRAME_SUPERPOSE * n_atoms * n_local / s / 1e9,
                                "fp64_peak_tflops_spec": FP64_PEAK_TFS,
                                "hbm_gbs": B_PER_ATOM_FRAME * n_atoms * n_local / s / 1e9}

    # -- aligned modes at N=1 (reported beside the headline) ------------------
    if wl.get("host"):
        out["stager"] = {"h2d_gbs": B_PER_ATOM_FRAME * n_atoms * n_local * a.steps / dt / 1e9,
                         "host_cache": bool(getattr(src, "cache", None) is not None),
                         "threads": a.stager_threads, "batch_frames": src.batch_frames,
                         "host_link_spec_gbs": 63.0}
        if wl.get("xtc"):
            out["stager"].update(xtc_decode=a.xtc_decode, xtc_cache=a.xtc_cache,
                                 xtc_bytes=os.path.getsize(xtc_path), xtc_write_s=t_w,
                                 xtc_frames_per_s=n_local * a.steps / dt,
                                 xtc_gb_per_s_compressed=os.path.getsize(xtc_path) * a.steps / dt / 1e9)
        out["roofline"]["note"] = "C5 is PCIe/host bound; the kernel roofline above is the device-side launch"
    if world == 1 and not a.no_modes and wl["align"] is None and not wl.get("host"):
        del traj, src
        torch.cuda.empty_cache()
        motion = motion_table(1, n_total)
        traj = generate(eng, n_atoms, b0, n_local, seed=0, motion=motion)
        torch.cuda.synchronize()
        src = DeviceSource(traj, offset=b0, n_traj=n_total)
        modes = {}
        for name, align in (("c3_frame0", "frame0"), ("rmsf_py_average", "average")):
            mdt, mt, _ = timed(align, a.mode_steps, 1)
            sweeps = 2 if align == "average" else 1
            sup = mt.ms("superpose")
            acc = mt.ms("accumulate")
            af = n_total * n_atoms * a.mode_steps / mdt
            modes[name] = {
                "atom_frames_per_s": af,
                "ms_per_step": mdt / a.mode_steps * 1e3,
                "sweeps": sweeps,
                "hbm_gbs_algorithmic": af * B_PER_ATOM_FRAME * sweeps / 1e9,
                "superpose_avg_ms": sum(sup) / len(sup),
                "superpose_gflops": FLOP_PER_ATOM_FRAME_SUPERPOSE * n_atoms * n_local / (sum(sup) / len(sup) / 1e3) / 1e9,
                "accumulate_avg_ms": sum(acc) / len(acc),
                "accumulate_hbm_gbs": B_PER_ATOM_FRAME * n_atoms * n_local / (sum(acc) / len(acc) / 1e3) / 1e9,
            }
        if cpu_c3 is not None:
            modes["c3_frame0"]["cpu_baseline"] = cpu_c3
        modes["c1_rmsf_py"] = c1_latency(eng, a.no_cpu_baseline)
        out["modes"] = modes
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
