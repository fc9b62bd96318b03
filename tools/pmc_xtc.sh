#!/bin/bash
# Instruction mix / wait cycles of the GPU XTC decoder (one rocprofv3 --pmc
# pass, 8 SQ counters), 250k-atom frames, N frames per launch (default 400).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
N=${1:-400}
export UB_KINDS=${UB_KINDS:-uniform}
TAG=${2:-pmc_xtc}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/$TAG -o run -- python3 tools/ubench_xtc.py $N > gpurun_out/$TAG.log 2>&1
echo rc=$?
python3 - "$TAG" <<'P'
import csv, glob, sys
for f in glob.glob(f'gpurun_out/{sys.argv[1]}/**/*counter_collection.csv', recursive=True):
    rows = list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if 'xtc_decode' in r['Kernel_Name']:
            agg.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(k, len(v), sum(v) / max(1, len(v)))
P
