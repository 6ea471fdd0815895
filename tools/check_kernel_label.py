"""Check that a bench line's roofline.kernel names the kernel rocprof timed.

    python tools/check_kernel_label.py gpurun_out/prof_c2

Reads <dir>/run_kernel_stats.csv (rocprofv3 --stats) and
<dir>/bench_under_rocprof.json (the bench line of the same run).  A plain
label (e.g. ``rt_trace_tiny<0,1,37>``) must be the template prefix of the
kernel with the most total time; a wavefront label (``wavefront
rt_trace_kernel<0,1,526> + 3 levels``) must name a level-0 kernel that ran
once per frame beside the level kernels.  Exit 1 on a mismatch."""
import csv
import json
import os
import sys


def norm(name: str) -> str:
    n = name.split("(", 1)[0].replace("void ", "").replace("rt::", "").replace(" ", "")
    return n


def main(d: str) -> int:
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    kernels = [(norm(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"])) for r in rows
               if not r["Name"].startswith("__amd")]
    with open(os.path.join(d, "bench_under_rocprof.json")) as f:
        label = json.load(f)["roofline"]["kernel"].replace(" ", "")
    if label.startswith("wavefront"):
        first = label[len("wavefront"):].split("+", 1)[0]
        ok = any(k.startswith(first[:-1] + ",") for k, _, _ in kernels)
        top = first
    else:
        top = max(kernels, key=lambda k: k[2])[0]
        ok = top.startswith(label[:-1] + ",")
    print(json.dumps({"dir": d, "label": label, "rocprof_top": top, "ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(max(main(d) for d in sys.argv[1:]))
