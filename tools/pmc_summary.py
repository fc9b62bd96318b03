"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

HBM bytes per dispatch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced streaming
reads (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for 16-B
stores.  The x2 is exact for k_welford_flat (dwordx4 loads); for dwordx3
loads it is uncalibrated (stated in the output)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read(d, counter):
    rows = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter:
                rows[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return rows


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def main(fetch_dir, write_dir, out=None, kernel=None, n_atoms=None, n_frames=None):
    fe, wr = read(fetch_dir, "FETCH_SIZE"), read(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fe) | set(wr), key=lambda k: -sum(fe.get(k, [0]))):
        f = fe.get(k, [])
        w = wr.get(k, [])
        fkb = sum(f) / len(f) if f else 0.0
        wkb = sum(w) / len(w) if w else 0.0
        res[short(k)] = {"dispatches": len(f), "fetch_kb_raw": fkb, "write_kb": wkb,
                         "hbm_bytes_corrected": 2 * fkb * 1024 + wkb * 1024}
    print(json.dumps(res, indent=1))
    if out:
        doc = {"kernels": res, "source": [fetch_dir, write_dir],
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                         "bytes = 2*FETCH_SIZE*1024 (gfx950 half-count of 16-B/lane reads) + WRITE_SIZE*1024"}
        if kernel:
            doc.update(kernel=kernel, n_atoms=int(n_atoms), n_frames=int(n_frames),
                       hbm_bytes_per_launch=res[kernel]["hbm_bytes_corrected"])
        json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    # pmc_summary.py FETCH_DIR WRITE_DIR [OUT.json KERNEL N_ATOMS N_FRAMES]
    main(*sys.argv[1:])
