"""Read-request bytes per dispatch from a rocprofv3 --pmc run of
TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_128B_sum, TCC_EA0_RDREQ_64B_sum and
TCC_EA0_RDREQ_32B_sum: bytes = 128 n128 + 64 n64 + 32 n32 (and the
remainder of RDREQ at 64 B, printed separately).  Diagnostic.

    python tools/calib/rdreq.py DIR [kernel-substring] [bytes-known]
"""
import collections
import csv
import glob
import json
import sys


def main(d, kernel="", known=0):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                per[(r["Kernel_Name"][:40], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in per.items():
        avg = {n: sum(v[1:] if len(v) > 2 else v) / len(v[1:] if len(v) > 2 else v) for n, v in c.items()}
        n = avg.get("TCC_EA0_RDREQ_sum", 0.0)
        n128 = avg.get("TCC_EA0_RDREQ_128B_sum", 0.0)
        n64 = avg.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        n32 = avg.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        b = 128 * n128 + 64 * n64 + 32 * n32
        e = {"rdreq": n, "n128": n128, "n64": n64, "n32": n32, "rest": n - n128 - n64 - n32, "bytes": b}
        if known:
            e["bytes_over_known"] = round(b / float(known), 4)
        out[f"{k[0]} grid={k[1]}"] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
