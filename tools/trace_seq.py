"""Per-launch durations of one repeating frame in a rocprofv3 kernel trace:
the dispatches from each launch of the frame's first kernel (default: the
level-0 trace kernel) to the next form a frame; prints, per position in the
frame, the kernel and its median duration (us) over the frames seen.

    python tools/trace_seq.py gpurun_out/x/run_kernel_trace.csv [first-kernel-substring]
"""
import csv
import json
import statistics
import sys


def main(path, first="rt_trace_kernel<0, 1, 526, false>"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if first in name:
            if cur:
                frames.append(cur)
            cur = []
        if cur is not None:
            cur.append((name.split("(")[0].replace("void ", "").replace("rt::", ""),
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                        int(r["Start_Timestamp"])))
    if cur:
        frames.append(cur)
    n = max(set(len(f) for f in frames), key=[len(f) for f in frames].count)
    frames = [f for f in frames if len(f) == n][1:]
    out = []
    for i in range(n):
        out.append({"pos": i, "kernel": frames[0][i][0], "median_us": round(statistics.median(f[i][1] for f in frames), 2)})
    span = statistics.median(f[-1][2] - f[0][2] for f in frames) / 1e3
    print(json.dumps({"frames": len(frames), "launches_per_frame": n, "first_to_last_start_us": round(span, 1),
                      "launches": out}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
