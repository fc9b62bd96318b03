"""Summarise tools/gpu_r6_pmc.sh's passes: per kernel family, per-dispatch
medians of each counter; read requests by size -> bytes (32/64/128 B)."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def load(d):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            did = r.get("Dispatch_Id", r.get("Correlation_Id"))
            c = per[k][r["Counter_Name"]]
            c[did] = c.get(did, 0.0) + float(r["Counter_Value"])
    return per


root = sys.argv[1]
for name in sorted(os.listdir(root)):
    d = os.path.join(root, name)
    if not os.path.isdir(d):
        continue
    per = load(d)
    print(f"== {name}")
    for k, cs in sorted(per.items(), key=lambda kv: -max(sum(v.values()) for v in kv[1].values())):
        if k.startswith("k_synth") or k.startswith("at::") or "elementwise" in k:
            continue
        med = {c: statistics.median(v.values()) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        extra = ""
        if "TCC_EA0_RDREQ_32B_sum" in med:
            b = 32 * med["TCC_EA0_RDREQ_32B_sum"] + 64 * med.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                128 * med.get("TCC_EA0_RDREQ_128B_sum", 0)
            extra = f"  -> read bytes (32/64/128-B requests) {b / 1e9:.3f} GB"
        if "WRITE_SIZE" in med:
            extra = f"  -> written {med['WRITE_SIZE'] * 1024 / 1e9:.3f} GB"
        vals = ", ".join(f"{c} {v:.4g}" for c, v in sorted(med.items()))
        print(f"  {k[:60]:60s} x{n}: {vals}{extra}")
