"""Per-kernel duration summary from a rocprofv3 --kernel-trace CSV, skipping
the first dispatch of each kernel and grid size (bench.py's stats-enabled, cold launch),
so the average matches bench.py's kernel_ms measured on the timed steps.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main(path):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        # per grid size too: synchronous renders into host memory launch the
        # kernel in row chunks (RT_OPT_HOST_CHUNK_MB), the timed steps whole
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        per[r["Kernel_Name"] + (f" grid={g}" if g else "")].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, v in per.items():
        w = v[1:] if len(v) > 2 else v
        out[k] = {"calls": len(v), "calls_summarised": len(w), "avg_us": round(statistics.mean(w), 3),
                  "median_us": round(statistics.median(w), 3), "min_us": round(min(w), 3),
                  "max_us": round(max(w), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
