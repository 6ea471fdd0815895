"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*counter_collection.csv)
per kernel: counter values averaged per dispatch of the trace kernel.

FETCH_SIZE / WRITE_SIZE are in KB.  Per MI355X_MICROARCH.md §HBM, on gfx950
FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming reads; this
kernel's reads are scalar loads of a ~1-3 MB scene, so both the raw and the x2
figure are printed and the write side (the RGBA8 framebuffer) dominates.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main(d="gpurun_out/pmc", kernel="rt_trace_kernel"):
    out = {}
    for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
        # the timed launches only: the non-counting instantiation (COUNT =
        # false) over the whole frame — not the counted launch, nor the row
        # chunks of synchronous renders into host memory (RT_OPT_HOST_CHUNK_MB)
        timed = [r for r in rows if "false>" in r["Kernel_Name"]] or rows
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
        # gfx950: FETCH_SIZE reads 1/2 of wide streamed reads (MI355X_MICROARCH.md
        # §HBM); the x2 is an upper bound here (this kernel's reads are scalar).
        out["hbm_bytes_per_launch"] = int(out["FETCH_SIZE"] * 1024 * 2 + out["WRITE_SIZE"] * 1024)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
