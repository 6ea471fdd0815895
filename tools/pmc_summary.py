"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*counter_collection.csv)
per kernel: counter values averaged per dispatch of the trace kernel.

FETCH_SIZE / WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports 1/2 of the
bytes of 16-B-per-lane vector reads but all of 64-B scalar loads
(tools/calib/fetch_calib.hip), so the traffic is taken from the read
requests by size (128 n128 + 64 n64 + 32 n32, calibrated to 0.15%) plus
WRITE_SIZE; the FETCH_SIZE x 2 upper bound is kept beside it.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(d="gpurun_out/pmc", kernel="rt::rt_trace_"):
    out = {}
    for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        # the timed launches only: the non-counting instantiation (COUNT =
        # false) over the whole frame — not the counted launch, nor the row
        # chunks of synchronous renders into host memory (RT_OPT_HOST_CHUNK_MB)
        # — of the kernel dispatched most (rt_trace_kernel, or the launch-camera
        # rt_trace_tiny<.., 37, ..> after its camera's first, mask-computing frame)
        timed = [r for r in rows if "false>" in r["Kernel_Name"]] or rows
        names = defaultdict(int)
        for r in timed:
            names[r["Kernel_Name"]] += 1
        if names:
            top = max(names, key=names.get)
            timed = [r for r in timed if r["Kernel_Name"] == top]
            out["kernel"] = top.split("(")[0]
        grid = max((int(r["Grid_Size"]) for r in timed), default=0)
        per = defaultdict(list)
        for r in timed:
            if int(r["Grid_Size"]) == grid:
                per[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in per.items():
            # skip the first (stats-enabled, cold) dispatch
            vals = v[1:] if len(v) > 1 else v
            out[k] = sum(vals) / len(vals)
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        # gfx950: FETCH_SIZE reads 1/2 of 16-B-per-lane vector reads
        # (MI355X_MICROARCH.md §HBM) but the exact bytes of 64-B scalar loads
        # (tools/calib/fetch_calib.hip), so x2 is only an upper bound here
        out["fetch_x2_bytes_per_launch"] = int(out["FETCH_SIZE"] * 1024 * 2 + out["WRITE_SIZE"] * 1024)
    if "TCC_EA0_RDREQ_128B_sum" in out and "WRITE_SIZE" in out:
        # calibrated (tools/calib: every pattern within 0.15% of its known
        # bytes): L2-to-fabric reads by request size, plus WRITE_SIZE (exact
        # for 4- and 16-B-per-lane stores); Infinity Cache hits included
        rd = (128 * out["TCC_EA0_RDREQ_128B_sum"] + 64 * out["TCC_EA0_RDREQ_64B_sum"] +
              32 * out.get("TCC_EA0_RDREQ_32B_sum", 0.0))
        out["read_bytes_per_launch"] = int(rd)
        out["hbm_bytes_per_launch"] = int(rd + out["WRITE_SIZE"] * 1024)
    elif "fetch_x2_bytes_per_launch" in out:
        out["hbm_bytes_per_launch"] = out["fetch_x2_bytes_per_launch"]
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
