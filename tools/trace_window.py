#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 kernel trace between two k_synth launches
(bench.py's modes each generate their frames first): which kernels a mode's
steps spend their device time in.

  python3 tools/trace_window.py <kernel_trace.csv> <first k_synth grid> [steps]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:80]


def main(argv):
    rows = sorted(csv.DictReader(open(argv[0])), key=lambda r: int(r["Start_Timestamp"]))
    grid0 = int(argv[1])
    steps = int(argv[2]) if len(argv) > 2 else 1
    start = next(i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_synth"
                 and int(r["Grid_Size_X"]) == grid0)
    i = start + 1
    while i < len(rows) and short(rows[i]["Kernel_Name"]) == "k_synth":
        i += 1
    end = next((j for j in range(i, len(rows)) if short(rows[j]["Kernel_Name"]) == "k_synth"), len(rows))
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in rows[i:end]:
        k = short(r["Kernel_Name"])
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    span = (int(rows[end - 1]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
    print(f"window: {end - i} launches, {span:.1f} us first start to last end, per step over {steps} steps:")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"  {k:80s} {cnt[k] / steps:6.1f} launches {tot[k] / steps:10.1f} us")
    print(f"  {'sum of kernel time':80s} {'':15s} {sum(tot.values()) / steps:10.1f} us")


if __name__ == "__main__":
    main(sys.argv[1:])
