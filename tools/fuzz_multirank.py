#!/usr/bin/env python3
"""Randomised parity sweep of the N > 1 pipeline (not product code, not a
test): P = 2..4 gloo ranks sharing the GPU, random atoms / selection /
frames / alignment / batch size, and merge slabs forced on where the flat
plan allows them -- each rank's RMSF against the oracle's mpirun -n P
emulation of RMSF.py.  ``--root``: half the cases merge with a reduce to a
random rank (merge_root); ``--planes``: half the shards are HBM coordinate
planes; ``--scatter``: a third of the other cases merge as a reduce-scatter
by atom slices with the RMSF gathered to a random root (merge_scatter);
``--exact``: half the unaligned cases run exact=True and must equal the
oracle's P-rank script bit for bit (``--exact-wide``: those with 4-6 ranks,
the default mpi4py reduce order, frames possibly fewer than ranks).
python tools/fuzz_multirank.py [n_cases [--root] [--planes] [--scatter] [--exact [--exact-wide]]]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mdanalysis-mpi_amd")
sys.path[:0] = [ROOT, PKG]

import numpy as np  # noqa: E402


def _worker(rank, size, init, q, case):
    sys.path[:0] = [ROOT, PKG]
    from datetime import timedelta

    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=size, timeout=timedelta(seconds=120))
    try:
        from rmsf_amd import parallel
        from rmsf_amd.engine import Engine
        from rmsf_amd.pipeline import run_pipeline
        from rmsf_amd.sources import DeviceSource, FrameList
        from rmsf_amd.synth import generate, motion_table
        eng = Engine(torch.device("cuda", 0))
        na, nf, align, sel, batch, slabs = (case[k] for k in ("na", "nf", "align", "sel", "batch", "slabs"))
        b0, b1 = parallel.blocks(nf, size)[rank]
        mt = motion_table(case["mseed"], nf) if align else None
        shard = generate(eng, na, b0, max(b1 - b0, 1), seed=case["seed"], motion=mt)[: b1 - b0]
        if case.get("planes"):  # the rank's shard as HBM coordinate planes, read in place
            src = DeviceSource(shard.transpose(1, 2).contiguous(), sel, offset=b0, n_traj=nf, layout="soa")
        else:
            src = DeviceSource(shard, sel, offset=b0, n_traj=nf)
        res = run_pipeline(eng, src, FrameList(nf), align=align, max_batch=batch, merge_slabs=slabs,
                           merge_root=case.get("root"), merge_scatter=bool(case.get("scatter")),
                           exact=bool(case.get("exact")))
        torch.cuda.synchronize()
        q.put((rank, None if res.rmsf is None else res.rmsf.cpu().numpy(), res.extras.get("merge_slabs", 0)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1))
    finally:
        dist.destroy_process_group()


def run_case(case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    d = tempfile.mkdtemp(prefix="fuzzmr_")
    init = "file://" + os.path.join(d, "store")
    ps = [ctx.Process(target=_worker, args=(r, case["P"], init, q, case), daemon=True) for r in range(case["P"])]
    for p in ps:
        p.start()
    try:
        return [q.get(timeout=240) for _ in ps]
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()


def main():
    from oracle import rmsf_oracle as O
    from oracle import synth as SY
    from rmsf_amd.synth import motion_table
    n_cases = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    rng = np.random.default_rng(303)
    worst, n_exact = 0.0, 0
    for k in range(n_cases):
        P = int(rng.integers(2, 5))
        big = k % 6 == 5  # every sixth case: 300k atoms, the chunk-aligned plan (merge slabs)
        na = 300_000 if big else int(rng.integers(1, 4000))
        nf = int(rng.integers(P, 40 if big else 160))
        align = None if big else [None, "frame0", "average"][int(rng.integers(0, 3))]
        if not big and rng.random() < 0.5:
            ns = int(rng.integers(1, na + 1))
            sel = np.sort(rng.choice(na, ns, replace=False))
        else:
            sel = None
        batch = None if (big or rng.random() < 0.5) else int(rng.integers(1, nf + 1))
        slabs = int(rng.integers(2, 5)) if big else None
        case = dict(P=P, na=na, nf=nf, align=align, sel=sel, batch=batch, slabs=slabs,
                    seed=int(rng.integers(0, 1000)), mseed=int(rng.integers(0, 1000)))
        if "--root" in sys.argv[2:] and rng.random() < 0.5:
            case["root"] = int(rng.integers(0, P))  # the merge as a reduce to this rank (RMSF.py:143)
        if "--planes" in sys.argv[2:] and rng.random() < 0.5:
            case["planes"] = True
        if "--scatter" in sys.argv[2:] and not case.get("planes") and rng.random() < 0.34:
            case["scatter"] = True  # reduce-scatter by atom slices, RMSF gathered to the root
            case["root"] = int(rng.integers(0, P))
        if "--exact" in sys.argv[2:] and align is None and not big and not case.get("scatter") and rng.random() < 0.5:
            case["exact"] = True  # RMSF.py's own arithmetic: bit for bit with the oracle's P-rank script
            if "--exact-wide" in sys.argv[2:]:
                # 4-6 ranks, where mpi4py's reduce tree and rank order differ
                # in bits; frames may be fewer than ranks (empty blocks)
                P = case["P"] = int(rng.integers(4, 7))
        out = run_case(case)
        if any(o[2] == -1 for o in out):
            print(f"case {k}: FAILED {[o[1] for o in out if o[2] == -1][:1]}", flush=True)
            sys.exit(1)
        traj = SY.frames(case["seed"], na, 0, nf, motion_table(case["mseed"], nf) if align else None,
                         atoms=None if not big else None)
        cols = np.arange(na) if sel is None else sel
        exp = (O.rmsf_script(traj, cols, None, size=P, align=align)["rmsf"] if not big
               else O.rmsf_two_pass(traj[:, cols]))
        root = case.get("root")
        if root is not None:  # only the root has a result
            assert all((o[1] is None) == (o[0] != root) for o in out), "reduce-to-root results on the wrong ranks"
        d = max(float(np.abs(o[1] - exp).max()) for o in out if o[1] is not None)
        if case.get("exact"):
            assert all(np.array_equal(o[1].view(np.uint64), exp.view(np.uint64)) for o in out if o[1] is not None), \
                f"case {k}: exact=True differs from the oracle's bits"
            n_exact += 1
        worst = max(worst, d)
        print(f"case {k:2d}: P={P} {na:7d} atoms {len(cols):7d} sel {nf:4d} frames align={align} "
              f"batch={batch} slabs={out[0][2]} root={root} planes={bool(case.get('planes'))} "
              f"scatter={bool(case.get('scatter'))} exact={bool(case.get('exact'))} max|d|={d:.2e}",
              flush=True)
        if d > 1e-6:
            print("EXCEEDS 1e-6", flush=True)
            sys.exit(1)
    print(f"all {n_cases} cases within 1e-6 A (worst {worst:.2e}); exact=True bit for bit in {n_exact} cases")


if __name__ == "__main__":
    main()
