"""For each bench JSON + rocprofv3 kernel-stats CSV of the same command:
the bench's per-launch HIP-event average for the roofline kernel against
rocprofv3's average for that kernel, and the roofline fraction (must be
<= 1).  Usage: roofline_vs_rocprof.py TAG NAME [NAME ...] (gpurun_out/TAG_NAME.json,
gpurun_out/TAG_NAME_rocprof/**/run_kernel_stats.csv)."""
import csv
import glob
import json
import sys


def main(tag, names):
    rows = []
    for n in names:
        b = json.load(open(f"gpurun_out/{tag}_{n}.json"))
        rf = b["roofline"]
        stats = glob.glob(f"gpurun_out/{tag}_{n}_rocprof/**/*kernel_stats.csv", recursive=True)
        best = None
        for r in csv.DictReader(open(stats[0])):
            name = r["Name"].replace("(anonymous namespace)::", "")
            short = name.replace("void ", "").split("<")[0].split("(")[0]
            if short == rf["kernel"] or short == rf["kernel"].rstrip("_sk") + "_sk":
                # the dominant instantiation: the one with the most total time
                if best is None or float(r["TotalDurationNs"]) > float(best["TotalDurationNs"]):
                    best = r
        roc = float(best["AverageNs"]) / 1e6 if best else None
        row = {"workload": n, "value": b["value"], "ms_per_step": b["ms_per_step"], "kernel": rf["kernel"],
               "bench_avg_launch_ms": rf["avg_launch_ms"], "rocprof_avg_ms": roc,
               "rocprof_kernel": best["Name"].split("(")[0].replace("void ", "") if best else None,
               "launches": rf["launches"], "frac": rf["frac"], "achieved_gbs": rf["achieved"]}
        if "stager" in b:
            row["h2d_gbs"] = b["stager"]["h2d_gbs"]
            row["h2d_bytes_per_step"] = b["stager"]["h2d_bytes_per_step"]
        rows.append(row)
        print(f"{n:10s} frac={rf['frac']:.3f} bench_avg={rf['avg_launch_ms']:.4f} ms rocprof_avg={roc if roc is None else round(roc, 4)} ms launches={rf['launches']}"
              + (f" h2d={row['h2d_gbs']:.1f} GB/s" if "h2d_gbs" in row else ""))
    return rows


if __name__ == "__main__":
    out = main(sys.argv[1], sys.argv[2:])
    json.dump(out, open(f"gpurun_out/{sys.argv[1]}_roofline_vs_rocprof.json", "w"), indent=1)
