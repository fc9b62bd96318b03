cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_fetch
for g in plain gather; do
  arg=""; [ $g = gather ] && arg="--gather"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch/$g -o run -- python3 tools/seq_once.py $arg > gpurun_out/pmc_fetch/$g.log 2>&1 || exit 1
  echo "$g done"
done
python3 - <<'P'
import csv, glob
for g in ("plain", "gather"):
    agg = {}
    for f in glob.glob(f"gpurun_out/pmc_fetch/{g}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_welford_seq" not in r["Kernel_Name"]:
                continue
            k = r.get("Dispatch_Id")
            agg[k] = agg.get(k, 0.0) + float(r["Counter_Value"])
    v = sorted(agg.values())
    print(g, "launches", len(v), "median FETCH_SIZE KB", v[len(v)//2], "-> GB x2 (gfx950 correction for wide reads not applied)", v[len(v)//2] * 1024 / 1e9)
P
