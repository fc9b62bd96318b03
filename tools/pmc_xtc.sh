cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export UB_KINDS=uniform
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_xtc -o run -- python3 tools/ubench_xtc.py 400 > gpurun_out/pmc_xtc.log 2>&1
echo rc=$?
python3 - <<'P'
import csv,glob
for f in glob.glob('gpurun_out/pmc_xtc/**/*counter_collection.csv', recursive=True):
    rows=list(csv.DictReader(open(f)))
    agg={}
    for r in rows:
        if 'xtc_decode' in r['Kernel_Name']:
            agg.setdefault(r['Counter_Name'],[]).append(float(r['Counter_Value']))
    for k,v in agg.items(): print(k, len(v), sum(v)/max(1,len(v)), v[:2])
P
