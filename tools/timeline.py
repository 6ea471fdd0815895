"""Print a window of a rocprofv3 kernel trace as a timeline (start, end,
duration in us, relative to the window's first kernel), starting at the
k-th launch of a kernel whose name contains --anchor.

    python tools/timeline.py gpurun_out/camtl_c3/run_kernel_trace.csv --anchor rt_trace_kernel --k 45 --n 14
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="rt_trace_kernel")
    ap.add_argument("--k", type=int, default=45)
    ap.add_argument("--n", type=int, default=14)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    s0 = idx[min(a.k, len(idx) - 1)]
    t0 = int(rows[s0]["Start_Timestamp"])
    for r in rows[s0:s0 + a.n]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:72]}")


if __name__ == "__main__":
    main()
