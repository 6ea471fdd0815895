"""Per-kernel averages of rocprofv3 --pmc CSVs (every kernel of the run, not
only the trace kernel as tools/pmc_summary.py): counter values averaged
over each kernel's dispatches, with VALU lane utilisation
(SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)), the mean waves resident
(SQ_WAVE_CYCLES / cycles) and the L2 hit rate where counted.

    python tools/pmc_kernels.py gpurun_out/pmcx_c3r > kernels.json
"""
import collections
import csv
import glob
import json
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, v in acc.items():
        m = {c: sum(x) / len(x) for c, x in v.items()}
        m["dispatches"] = max(len(x) for x in v.values())
        if m.get("SQ_ACTIVE_INST_VALU"):
            m["lane_util"] = round(m.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * m["SQ_ACTIVE_INST_VALU"]), 3)
        if m.get("SQ_WAVE_CYCLES"):
            m["wait_share"] = round(m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"], 3)
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            tot = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            m["l2_hit_rate"] = round(m["TCC_HIT_sum"] / tot, 3) if tot else None
        out[k] = {c: (round(x, 3) if isinstance(x, float) else x) for c, x in m.items()}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
