#!/usr/bin/env python3
"""HBM-resident coordinate planes (DeviceSource(layout="soa"): each batch
gathered into (frame, atom, xyz) rows by rmsf_gather_planes) against the
row layout read in place, 100k atoms x 20k frames, no alignment and C3's
frame-0 alignment: ms per run_pipeline call (median of 5) and whether the
RMSF agrees.  python tools/time_device_soa.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mdanalysis-mpi_amd")]

import torch  # noqa: E402

from rmsf_amd.engine import Engine  # noqa: E402
from rmsf_amd.pipeline import run_pipeline  # noqa: E402
from rmsf_amd.sources import DeviceSource, FrameList  # noqa: E402
from rmsf_amd.synth import generate, motion_table  # noqa: E402


def main():
    eng = Engine()
    n, nf = 100_000, 20_000
    for align in (None, "frame0"):
        rows = generate(eng, n, 0, nf, seed=0, motion=motion_table(1, nf) if align else None)
        planes = rows.transpose(1, 2).contiguous()  # [F, 3, n]
        fl = FrameList(nf)
        out = {}
        for name, src in (("rows", DeviceSource(rows)), ("planes", DeviceSource(planes, layout="soa"))):
            run_pipeline(eng, src, fl, align=align)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                r = run_pipeline(eng, src, fl, align=align).rmsf
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e3)
            out[name] = (sorted(ts)[2], r)
        d = float((out["rows"][1] - out["planes"][1]).abs().max())
        print(f"align={align}: rows {out['rows'][0]:.2f} ms, planes {out['planes'][0]:.2f} ms "
              f"({out['planes'][0] / out['rows'][0]:.2f}x), max|d rmsf| {d:.2e}", flush=True)
        del rows, planes
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
