"""Few-frame worst-case parity sweep of the ALIGNED path (round 6, verdict
item 1; not product code, not a test).

Where one f32 rounding flip of an aligned coordinate (RMSF.py:99-101 /
133-135) weighs most -- 2, 4, 8 and 10 frames -- every (selection shape,
align mode, frame count) group runs N_SEEDS seeded trajectories through
  * the frame-parallel path, RMSF(x, align=..., exact=False): max |dRMSF|
    and max |daverage| against the oracle's restatement of RMSF.py;
  * exact=True: must equal the restatement bit for bit (mismatch count).
The oracle runs in a spawned CPU process pool beside the GPU work.  One
line per group; the table is committed under profiles/.

    python tools/fuzz_fewframes.py [n_seeds] [--quick]
    FUZZ_FRAMES=256,384,512 python tools/fuzz_fewframes.py 20   (other frame counts)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402

# (label, n_atoms, n_sel, masses): RMSF.py's own shape (214 CA of 47,681),
# denser CA-like selections, and whole large systems
SHAPES = [("214 of 47,681 (RMSF.py)", 47_681, 214, "ca"),
          ("2,000 of 47,681", 47_681, 2_000, "ca"),
          ("20,000 of 100,000", 100_000, 20_000, None),
          ("200,000 of 200,000", 200_000, 200_000, None)]
FRAMES = (2, 4, 8, 10)
if os.environ.get("FUZZ_FRAMES"):  # e.g. "256,384,512": the bound's side of AUTO_EXACT_FRAMES
    FRAMES = tuple(int(x) for x in os.environ["FUZZ_FRAMES"].split(","))
ALIGNS = ("frame0", "average")


def case_inputs(n_atoms, n_sel, masses, nf, seed):
    from make_golden import motion_table
    from oracle import synth as SY
    traj = SY.frames(1000 + seed, n_atoms, 0, nf, motion_table(2000 + seed, nf))
    rng = np.random.default_rng(3000 + seed)
    sel = np.arange(n_atoms) if n_sel == n_atoms else np.sort(rng.choice(n_atoms, n_sel, replace=False))
    m = np.full(n_sel, 12.011) if masses == "ca" else None
    return traj, sel, m


def oracle_job(args):
    n_atoms, n_sel, masses, nf, seed, align = args
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
    from oracle import rmsf_oracle as O
    traj, sel, m = case_inputs(n_atoms, n_sel, masses, nf, seed)
    r = O.rmsf_script(traj, sel, m, size=1, align=align)
    return r["rmsf"], (r["average"] if align == "average" else None)


def main():
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import multiprocessing as mp

    import torch

    from rmsf_amd import RMSF
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 50
    quick = "--quick" in sys.argv
    shapes = SHAPES[:2] if quick else SHAPES
    if os.environ.get("FUZZ_SHAPES"):  # e.g. "2,3": a subset, to split a long sweep over calls
        shapes = [SHAPES[int(i)] for i in os.environ["FUZZ_SHAPES"].split(",")]
    workers = min(16, len(os.sched_getaffinity(0)))
    pool = mp.get_context("spawn").Pool(workers)
    print(f"# tools/fuzz_fewframes.py: {n_seeds} seeds per group, oracle on {workers} CPU processes", flush=True)
    print("# group | seeds | default max|dRMSF| | default max|davg| | default cases > 1e-6 A | exact bitwise mismatches",
          flush=True)
    worst, over, mism, total = 0.0, 0, 0, 0
    for label, na, ns, ms in shapes:
        for align in ALIGNS:
            for nf in FRAMES:
                t0 = time.time()
                jobs = [(na, ns, ms, nf, s, align) for s in range(n_seeds)]
                pending = pool.map_async(oracle_job, jobs)
                dmax = amax = 0.0
                n_over = n_mis = 0
                got = []
                for s in range(n_seeds):
                    traj, sel, m = case_inputs(na, ns, ms, nf, s)
                    x = torch.tensor(traj, device="cuda")
                    d = RMSF(x, select=sel, masses=m, align=align, exact=False).run().results
                    e = RMSF(x, select=sel, masses=m, align=align, exact=True).run().results
                    got.append((d.rmsf, d.get("average"), e.rmsf, e.get("average")))
                    del x
                want = pending.get(timeout=1800)
                for (dr, da, er, ea), (wr, wa) in zip(got, want):
                    dd = float(np.abs(dr - wr).max())
                    dmax = max(dmax, dd)
                    n_over += dd > 1e-6
                    if wa is not None:
                        amax = max(amax, float(np.abs(da - wa).max()))
                    bad = not np.array_equal(er.view(np.uint64), wr.view(np.uint64))
                    if wa is not None:
                        bad |= not np.array_equal(ea.view(np.uint64), wa.view(np.uint64))
                    n_mis += bad
                worst = max(worst, dmax)
                over += n_over
                mism += n_mis
                total += n_seeds
                print(f"{label:26s} {align:7s} {nf:2d} frames | {n_seeds} | {dmax:.3e} | "
                      f"{amax:.3e} | {n_over} | {n_mis}   ({time.time() - t0:.1f} s)", flush=True)
    pool.close()
    print(f"# {total} cases: default path worst {worst:.3e} A, {over} cases over 1e-6 A; "
          f"exact=True bit for bit in {total - mism} of {total}", flush=True)


if __name__ == "__main__":
    main()
