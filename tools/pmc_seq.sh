#!/bin/bash
# Where k_welford_seq's time goes (exact=True at C2): effective clock and
# VALU / wait shares from separate rocprofv3 --pmc passes over
# tools/seq_once.py (5 launches of 100k x 20k; nothing else traced).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_seq
timeout -k 10 120 python3 tools/seq_once.py > gpurun_out/pmc_seq/plain.txt 2>&1 || exit 1
i=0
for set in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_seq/p$i -o run \
      -- python3 tools/seq_once.py > gpurun_out/pmc_seq/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_seq/p$i.log; exit $rc; }
done
python3 - <<'P'
import csv, glob
agg = {}
for f in glob.glob("gpurun_out/pmc_seq/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_welford_seq" not in r["Kernel_Name"]:
            continue
        d = agg.setdefault(r["Counter_Name"], {})
        k = r.get("Dispatch_Id", r.get("Correlation_Id"))
        d[k] = d.get(k, 0.0) + float(r["Counter_Value"])
for c, v in sorted(agg.items()):
    vals = sorted(v.values())
    print(f"{c:24s} launches {len(vals)}  median per launch {vals[len(vals) // 2]:.6g}")
P
