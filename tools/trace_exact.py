"""Per-launch timeline of the exact aligned path's kernels from a rocprofv3
kernel-trace CSV (tools/gpu_r6_exprof.sh): start (us from the first launch),
duration, stream, kernel, grid -- the last N launches.
  python tools/trace_exact.py gpurun_out/<dir>/prof/run_kernel_trace.csv [N]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
keep = [r for r in rows if re.search(r"k_seq|k_ref|k_accum_seq", r["Kernel_Name"])]
t0 = int(keep[-n]["Start_Timestamp"]) if len(keep) >= n else int(keep[0]["Start_Timestamp"])
for r in keep[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(anonymous namespace\)::|void |\(.*", "", r["Kernel_Name"])
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f} us  stream {r['Stream_Id']:>2}  {name:42s} "
          f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")
