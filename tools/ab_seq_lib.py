#!/usr/bin/env python3
"""A/B of rmsf_welford_sequential (k_welford_seq, exact=True) between two
builds of the library in one process: tools/_ab/librmsf_old.so and the
current one.  HIP-event medians of alternating rounds at 100k x 20k
(contiguous) and 100k-of-120k atoms (gathered); (mean, sumsquares) compared
bit for bit there, on ragged frame counts / nonzero k0, and on frames with
zeros, infinities and NaN (the per-block slow path), all rows and a
gathered selection.
  python tools/ab_seq_lib.py [--old LIB] [--new LIB] [--reps 7]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import LIB_PATH, SIGNATURES  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate  # noqa: E402


def lib(path):
    L = ctypes.CDLL(path)
    for name in ("rmsf_welford_sequential", "rmsf_welford_sequential_workspace_bytes"):
        f = getattr(L, name)
        f.restype, f.argtypes = SIGNATURES[name]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--old", default=os.path.join(ROOT, "tools", "_ab", "librmsf_old.so"))
    ap.add_argument("--new", default=LIB_PATH)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--shapes", action="store_true", help="a sweep of selection sizes and densities instead")
    a = ap.parse_args()
    libs = {"old": lib(a.old), "new": lib(a.new)}
    eng = Engine()
    s = eng.stream

    def call(L, traj, fstride, nf, n_sel, sel, k0, m, q, work):
        rc = L.rmsf_welford_sequential(traj.data_ptr(), fstride, nf, n_sel, None if sel is None else sel.data_ptr(),
                                       k0, m.data_ptr(), q.data_ptr(), work.data_ptr(), work.numel() * 8, s)
        assert rc == 0, rc

    def bits(t):
        return t.cpu().numpy().view(np.uint64)

    def same_bits(a, b):
        """bit for bit, NaN payloads aside (the NaN pattern must match; as
        tests/test_gpu_exact.py compares specials)"""
        fa, fb = a.view(np.float64), b.view(np.float64)
        na, nb = np.isnan(fa), np.isnan(fb)
        return bool(np.array_equal(na, nb) and np.array_equal(a[~na], b[~nb]))

    ok = True
    cases = (("contiguous 100k", 100_000, 100_000, 20_000),
             ("gathered 100k of 120k", 120_000, 100_000, 20_000),
             ("sparse (CA-like) 20k of 300k", 300_000, 20_000, 5_000))
    if a.shapes:
        cases = (("dense 20k of 24k", 24_000, 20_000, 20_000), ("dense 50k of 60k", 60_000, 50_000, 10_000),
                 ("contiguous 20k", 20_000, 20_000, 20_000), ("contiguous 50k", 50_000, 50_000, 10_000),
                 ("third 100k of 300k", 300_000, 100_000, 4_000), ("sparse 100k of 1.5M", 1_500_000, 100_000, 800),
                 ("sparse 50k of 750k", 750_000, 50_000, 1_600), ("half 200k of 400k", 400_000, 200_000, 3_000))
    for label, n_atoms, n_sel, nf in cases:
        traj = generate(eng, n_atoms, 0, nf, seed=0)
        sel = None if n_sel == n_atoms else eng.sel_tensor(np.sort(np.random.default_rng(1).choice(
            n_atoms, n_sel, replace=False)))
        work = eng.empty(libs["new"].rmsf_welford_sequential_workspace_bytes(nf) // 8 + 2)
        out = {k: (eng.empty(3 * n_sel), eng.empty(3 * n_sel)) for k in libs}
        t = {k: [] for k in libs}
        for k in libs:
            call(libs[k], traj, 3 * n_atoms, nf, n_sel, sel, 0, *out[k], work)
        torch.cuda.synchronize()
        for _ in range(a.reps):
            for k in libs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                call(libs[k], traj, 3 * n_atoms, nf, n_sel, sel, 0, *out[k], work)
                e1.record()
                torch.cuda.synchronize()
                t[k].append(e0.elapsed_time(e1))
        same = all(np.array_equal(bits(out["old"][i]), bits(out["new"][i])) for i in (0, 1))
        ok &= same
        o, n = float(np.median(t["old"])), float(np.median(t["new"]))
        print(f"{label} x {nf}: old {o:.3f} ms ({12 * n_sel * nf / (o / 1e3) / 1e9 / 8000:.3f} of 8 TB/s)  "
              f"new {n:.3f} ms ({12 * n_sel * nf / (n / 1e3) / 1e9 / 8000:.3f})  {(n / o - 1) * 100:+.1f} %  "
              f"bits equal {same}", flush=True)
        print(f"   old [{' '.join(f'{x:.3f}' for x in t['old'])}]\n   new [{' '.join(f'{x:.3f}' for x in t['new'])}]",
              flush=True)
        del traj, work
        torch.cuda.empty_cache()
    if a.shapes:
        print("full-size shapes bit-equal:", ok, flush=True)
        return 0 if ok else 1
    # ragged frame counts, nonzero k0, continuing state; then special values
    traj = generate(eng, 5000, 0, 700, seed=3)
    h = traj.cpu().numpy()
    rng = np.random.default_rng(5)
    hs = h.copy().reshape(700, -1)
    for val in (0.0, -0.0, np.inf, -np.inf, np.nan):
        idx = rng.choice(hs.size, 40, replace=False)
        hs.reshape(-1)[idx] = val
    trajs = torch.tensor(hs.reshape(h.shape), device=eng.device)
    work = eng.empty(libs["new"].rmsf_welford_sequential_workspace_bytes(700) // 8 + 2)
    gsel = eng.sel_tensor(np.sort(rng.choice(5000, 1777, replace=False)))
    for name, tr in (("plain", traj), ("zeros/inf/nan", trajs)):
        for sl, ns in ((None, 5000), (gsel, 1777)):
            for nf2, k0 in ((1, 0), (7, 0), (8, 0), (15, 3), (16, 0), (17, 9), (31, 5), (33, 64), (129, 1000),
                            (700, 3), (700, 0)):
                res = {}
                for k in libs:
                    mm = torch.tensor(np.full(3 * ns, 50.0), device=eng.device)
                    qq = torch.tensor(np.full(3 * ns, 1.0), device=eng.device)
                    call(libs[k], tr, 3 * 5000, nf2, ns, sl, k0, mm, qq, work)
                    torch.cuda.synchronize()
                    res[k] = (bits(mm), bits(qq))
                same = all(same_bits(res["old"][i], res["new"][i]) for i in (0, 1))
                ok &= same
                if not same:
                    print(f"  DIFF {name} sel={'yes' if sl is not None else 'no'} nf={nf2} k0={k0}", flush=True)
    print("ragged / special shapes all bit-equal:", ok, flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
