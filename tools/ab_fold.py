#!/usr/bin/env python3
"""A/B of the balanced grid's plan walks between two builds of the library in
one process (tools/_ab/librmsf_old.so vs the current one): the fold
(rmsf_fold_balanced / _shift, k_fold_sk), the accumulate and the
superposition (k_frame_stats + k_qcp_frames) at the strong-scaling shares,
each launch timed alone with HIP events, A/B/A; outputs compared byte for
byte, per buffer.  python tools/ab_fold.py [--old LIB] [--new LIB]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rmsf_amd._lib import LIB_PATH, RMSF_MODE_WELFORD, SIGNATURES  # noqa: E402
from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def lib(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
    return L


def refold(wk, j):
    """k_fold_sk's walk and Chan fold for coordinate j, in Python floats."""
    h = wk[:16].view(np.int64)
    lanes, C, nf, T, G, P, cpl, mode, S, cw = (int(v) for v in h[:10])
    p0 = wk[16:]
    slot_d = cw * cpl
    p1 = G * P * slot_d
    c = (j // cpl) // cw
    off = j - c * slot_d
    clo, chi = c * nf, c * nf + nf

    def sk_lo(b):
        return T * b // G

    def seg_len(lo, hi):
        f0 = lo - (lo // nf) * nf
        return min(hi - lo, nf - f0, 4096)

    b = clo * G // T
    while b > 0 and sk_lo(b) > clo:
        b -= 1
    while sk_lo(b + 1) <= clo:
        b += 1
    lo, hi, slot = sk_lo(b), sk_lo(b + 1), b * P
    while lo < clo:
        lo += seg_len(lo, hi)
        slot += 1
    segs = []
    while True:
        if lo >= hi:
            b += 1
            if b >= G:
                break
            lo, hi, slot = sk_lo(b), sk_lo(b + 1), b * P
        if lo >= chi:
            break
        ln = float(seg_len(lo, hi))
        segs.append((slot, ln, float(p0[slot * slot_d + off]), float(p0[p1 + slot * slot_d + off])))
        lo += int(ln)
        slot += 1
    mu, M = chan(segs)
    return mu, M, segs


def chan(segs, ops=None):
    """Chan's merge of (slot, n, mean, M2) in list order; ops = (mul, add, sub, div) to evaluate elsewhere."""
    mul, add, sub, div = ops or ((lambda a, b: a * b), (lambda a, b: a + b), (lambda a, b: a - b), (lambda a, b: a / b))
    n1, mu, M = 0.0, 0.0, 0.0
    for _, ln, pm, pq in segs:
        if n1 <= 0:
            mu, M = pm, pq
        else:
            t = n1 + ln
            d = sub(pm, mu)
            mun = div(add(mul(n1, mu), mul(ln, pm)), t)
            M = add(add(M, pq), mul(div(n1 * ln, t), mul(d, d)))
            mu = mun
        n1 = ln if n1 <= 0 else n1 + ln
    return float(mu), float(M)


def gpu_ops():
    """The same f64 operations as single-element torch kernels on the GPU."""
    T = lambda v: v if torch.is_tensor(v) else torch.tensor(v, dtype=torch.float64, device="cuda")  # noqa: E731
    return ((lambda a, b: T(a) * T(b)), (lambda a, b: T(a) + T(b)), (lambda a, b: T(a) - T(b)),
            (lambda a, b: T(a) / T(b)))


def med_time(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--old", default=os.path.join(ROOT, "tools", "_ab", "librmsf_old.so"))
    ap.add_argument("--new", default=LIB_PATH)
    ap.add_argument("--dump", help="write the differing coordinates' segments (n, mean, M2) as JSON")
    a = ap.parse_args()
    print("old", a.old, "new", a.new, flush=True)
    libs = {"old": lib(a.old), "new": lib(a.new)}
    dump = []
    eng = Engine()
    s = lambda: eng.stream  # noqa: E731
    for n, nf, aligned in ((100_000, 2_500, False), (100_000, 20_000, False), (1_000_000, 2_500, False),
                           (100_000, 2_500, True), (100_000, 20_000, True)):
        traj = generate(eng, n, 0, nf, seed=0, motion=motion_table(1, nf) if aligned else None)
        nc = 3 * n
        ref, info = eng.reference_setup(n, frame_ptr=traj.data_ptr())
        xf = {k: eng.zeros(nf, 16) for k in libs}
        sw = eng.empty(eng.workspace_bytes(n, nf) // 8 + 2)
        work = eng.empty(eng.balanced_workspace_bytes(n, nf) // 8 + 2)
        shift = traj[0].reshape(-1).clone()
        out = {k: [eng.zeros(nc), eng.zeros(nc), eng.zeros(2 * nc)] for k in libs}
        t = {k: {"superpose": [], "accumulate": [], "fold": []} for k in libs}
        parts = {}
        for order in ("old", "new", "old", "new"):
            L = libs[order]

            def sup():
                assert L.rmsf_superpose(traj.data_ptr(), nc, nf, n, None, None, ref.data_ptr(), info.data_ptr(),
                                        xf[order].data_ptr(), sw.data_ptr(), sw.numel() * 8, s()) == 0

            x = xf[order].data_ptr() if aligned else None
            ip = info.data_ptr() if aligned else None

            def acc():
                assert L.rmsf_accumulate_balanced(traj.data_ptr(), nc, nf, n, None, x, ip, RMSF_MODE_WELFORD, 0,
                                                  work.data_ptr(), work.numel() * 8, s()) == 0

            a0, a1, tt = out[order]

            def fold():
                assert L.rmsf_fold_balanced_shift(work.data_ptr(), nc, 0, a0.data_ptr(), a1.data_ptr(),
                                                  shift.data_ptr(), 1, None, tt.data_ptr(), s()) == 0

            reps = 30 if nf <= 2500 else 10
            if aligned:
                t[order]["superpose"] += med_time(sup, reps)
            sup()
            acc()
            torch.cuda.synchronize()
            t[order]["accumulate"] += med_time(acc, reps)
            t[order]["fold"] += med_time(fold, reps)  # acc_n = 0: the fold is idempotent
            acc()
            fold()
            torch.cuda.synchronize()
            parts[order] = work.cpu().numpy()
        eq = [np.array_equal(a.cpu().numpy().view(np.uint64), b.cpu().numpy().view(np.uint64))
              for a, b in zip(out["old"] + [xf["old"]], out["new"] + [xf["new"]])]
        same = all(eq)
        if not same:
            diffs = [float((a - b).abs().max()) for a, b in zip(out["old"] + [xf["old"]], out["new"] + [xf["new"]])]
            same = f"False (mean, M2, T, xform equal: {eq}; max |diff| {diffs})"
            if not eq[0]:
                # which build is IEEE-exact: refold the differing coordinates
                # from each build's own partials in Python f64 (same walk, same order)
                po, pn = parts["old"], parts["new"]
                print(f"    partials equal {np.array_equal(po.view(np.uint64), pn.view(np.uint64))}", flush=True)
                mo, mn = out["old"][0].cpu().numpy(), out["new"][0].cpu().numpy()
                for j in np.flatnonzero(mo != mn)[:3]:
                    ro, _, segs = refold(po, int(j))
                    rn = refold(pn, int(j))[0]
                    print(f"    coord {j}: old {mo[j]!r} (python on its partials {ro!r}) new {mn[j]!r} "
                          f"(python {rn!r})", flush=True)
                    print(f"      segments (slot, n): {[(s_[0], s_[1]) for s_ in segs]}; "
                          f"torch-on-GPU ops {chan(segs, gpu_ops())[0]!r}; "
                          f"reversed order {chan(segs[::-1])[0]!r}", flush=True)
                    dump.append({"case": [n, nf, aligned], "coord": int(j), "old": float(mo[j]), "new": float(mn[j]),
                                 "old_m2": float(out["old"][1][j]), "new_m2": float(out["new"][1][j]),
                                 "segs": [[int(a), b, c, d] for a, b, c, d in segs]})
                    import itertools
                    hits = [p for p in itertools.permutations(range(len(segs)))
                            if len(segs) <= 7 and chan([segs[i] for i in p])[0] in (mo[j], mn[j])]
                    print(f"      orders giving old/new: {[(p, chan([segs[i] for i in p])[0] == mo[j]) for p in hits[:6]]}",
                          flush=True)
        line = f"{n:8d} x {nf:6d} aligned {aligned!s:5s}:"
        for kname in ("superpose", "accumulate", "fold"):
            if not t["old"][kname]:
                continue
            o, w = float(np.median(t["old"][kname])), float(np.median(t["new"][kname]))
            line += f"  {kname} old {o:8.1f} new {w:8.1f} us ({(w / o - 1) * 100:+.1f} %)"
        print(line + f"  bitwise equal {same}", flush=True)
        del traj, work, sw
        torch.cuda.empty_cache()
    if a.dump and dump:
        import json
        with open(a.dump, "w") as f:
            json.dump(dump, f)


if __name__ == "__main__":
    main()
