#!/usr/bin/env python3
"""Recompute bench.py's roofline from the rocprofv3 run of the SAME command.

  python3 tools/roofline_vs_rocprof.py <rocprof dir> <bench log> [--out json]

<rocprof dir> holds ``*_kernel_stats.csv`` and ``*_kernel_trace.csv`` of
``rocprofv3 --kernel-trace --stats -- python3 bench.py ...``; <bench log> is
that run's stdout (its JSON line).  For the line's dominant kernel
(``roofline.kernel``) it reports

  * the stats CSV average over every launch of that kernel name (warm-up
    and later modes included: since round 5 the C4-share and C5 modes launch
    the same kernel at other sizes) and the trace-derived average of the
    headline's timed launches: the kernel's launches [warmup, warmup +
    steps) in trace order (the headline runs first in bench.py);
  * frac recomputed from each as algorithmic bytes per launch (the line's
    ``algorithmic_bytes_per_launch``: 12 B per atom-frame)
    / duration / 8 TB/s, against the line's own frac (HIP events);
  * whether the kernel average stays under the same run's ``ms_per_step``.

Checks (exit status 1 if either fails): the recomputed frac (timed launches)
within 2 % of the line's, and the kernel average <= ms_per_step.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys

PEAK_GBS = 8000.0


def json_line(path: str) -> dict:
    for line in reversed(open(path, errors="replace").read().splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def one(pattern: str) -> str:
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"nothing matches {pattern}")
    return hits[0]


def main(argv):
    if len(argv) < 2:
        raise SystemExit(__doc__)
    prof, log = argv[0], argv[1]
    out_path = argv[argv.index("--out") + 1] if "--out" in argv else None
    line = json_line(log)
    rf = line["roofline"]
    kern, steps = rf["kernel"], int(line["steps"])
    bytes_launch = float(rf["algorithmic_bytes_per_launch"])

    stats = None
    for row in csv.DictReader(open(one(os.path.join(prof, "**", "*kernel_stats.csv")))):
        if f"{kern}<" in row["Name"] or row["Name"].split("(")[0].endswith(kern):
            stats = row
            break
    if stats is None:
        raise SystemExit(f"{kern} not in the stats CSV")
    launches = []
    for row in csv.DictReader(open(one(os.path.join(prof, "**", "*kernel_trace.csv")))):
        if row["Kernel_Name"] == stats["Name"]:
            launches.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    launches.sort()
    warm = int(line["warmup"])
    timed = launches[warm:warm + steps]
    avg_all_ms = float(stats["AverageNs"]) / 1e6
    avg_timed_ms = sum(b - a for a, b in timed) / len(timed) / 1e6
    frac = lambda ms: bytes_launch / (ms / 1e3) / 1e9 / PEAK_GBS  # noqa: E731
    res = {
        "kernel": stats["Name"],
        "line": {"value": line["value"], "ms_per_step": line["ms_per_step"], "steps": steps,
                 "avg_launch_ms": rf["avg_launch_ms"], "frac": rf["frac"], "achieved_gbs": rf["achieved"]},
        "rocprof_stats": {"calls": int(stats["Calls"]), "avg_ms": avg_all_ms, "min_ms": float(stats["MinNs"]) / 1e6,
                          "max_ms": float(stats["MaxNs"]) / 1e6, "frac": frac(avg_all_ms)},
        "rocprof_timed_launches": {"n": len(timed), "which": f"launches {warm}..{warm + steps - 1} of the kernel in "
                                                             "trace order (the headline's timed region)",
                                   "avg_ms": avg_timed_ms, "frac": frac(avg_timed_ms)},
        "algorithmic_bytes_per_launch": bytes_launch,
    }
    rel = abs(res["rocprof_timed_launches"]["frac"] - rf["frac"]) / rf["frac"]
    res["frac_rel_diff_timed_vs_line"] = rel
    res["frac_rel_diff_stats_vs_line"] = abs(res["rocprof_stats"]["frac"] - rf["frac"]) / rf["frac"]
    res["kernel_avg_le_ms_per_step"] = avg_timed_ms <= line["ms_per_step"]
    res["ok"] = rel <= 0.02 and res["kernel_avg_le_ms_per_step"]
    text = json.dumps(res, indent=1)
    print(text)
    if out_path:
        open(out_path, "w").write(text + "\n")
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
