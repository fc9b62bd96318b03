#!/bin/bash
# fp64 VALU work of the aligned sweep's kernels (C3: 100k atoms x 20k frames,
# 2 timed steps): ONE rocprofv3 --pmc pass of 7 SQ counters, nothing else
# traced.  FLOPs per launch = (FMA_F64 * 2 + ADD_F64 + MUL_F64) * 64 lanes
# (rocprofv3's TOTAL_64_OPS without the int64 term), against SURVEY 8(d)'s
# algorithmic 27 flop per atom-frame for the superposition sums.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-pmc_flops}
WL=${2:-c3}    # c2 (flat Welford), c3 (superposition + aligned Welford), average (+ the aligned sum)
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
    SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES --output-format csv -d gpurun_out/$TAG -o run \
    -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --no-modes > gpurun_out/$TAG.log 2>&1
rc=$?; echo rc=$rc; if [ $rc -ne 0 ]; then tail -5 gpurun_out/$TAG.log; exit $rc; fi
python3 - "$TAG" <<'P'
import csv, glob, json, sys
tag = sys.argv[1]
agg = {}
for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        for base in ("k_frame_stats", "k_accum_split_sk", "k_qcp_frames", "k_welford_flat_sk", "k_fold_sk"):
            if base in k:
                # the template arguments tell the sweeps apart (<0,...> Welford, <1,...> sum)
                key = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
                d = agg.setdefault(key, {})
                d.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), 0.0)
                d[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
out = {}
af = 100_000 * 20_000
for key, d in agg.items():
    per = {c: sum(v.values()) / max(1, len(v)) for c, v in d.items()}
    launches = max(len(v) for v in d.values())
    fl = (2 * per.get("SQ_INSTS_VALU_FMA_F64", 0) + per.get("SQ_INSTS_VALU_ADD_F64", 0)
          + per.get("SQ_INSTS_VALU_MUL_F64", 0)) * 64
    out[key] = {"launches": launches, "per_launch": per, "fp64_flop_per_launch": fl,
                "fp64_flop_per_atom_frame": fl / af, "valu_insts_per_atom_frame_wave64": per.get("SQ_INSTS_VALU", 0) * 64 / af}
    print(key, launches, {c: f"{v:.4g}" for c, v in per.items()}, f"flop/atom-frame {fl / af:.2f}")
json.dump(out, open(f"gpurun_out/{tag}.json", "w"), indent=1)
P
