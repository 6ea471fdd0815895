"""Collect per-config PMC summaries (tools/pmc_summary.py output) into
profiles/pmc.json, the file bench.py reads its measured HBM bytes and VALU
instruction counts from.

    python tools/pmc_collect.py profiles/r01/session2 c2 c3 c5 c4s9
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import product_src_sha256  # noqa: E402


def main(src, *configs):
    out_path = os.path.join(REPO, "profiles", "pmc.json")
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for c in configs:
        f = os.path.join(src, f"pmc_{c}_summary.json")
        d = json.load(open(f))
        out[f"{c}_n1"] = {"hbm_bytes_per_launch": d.get("hbm_bytes_per_launch"),
                          "fetch_x2_bytes_per_launch": d.get("fetch_x2_bytes_per_launch"),
                          "SQ_INSTS_VALU": d.get("SQ_INSTS_VALU"), "SQ_INSTS_SALU": d.get("SQ_INSTS_SALU"),
                          "SQ_WAVES": d.get("SQ_WAVES"), "source": os.path.relpath(f, REPO),
                          "src_sha256": product_src_sha256()}
    out["_note"] = ("Per timed rt_trace_kernel launch, from rocprofv3 --pmc passes (one counter group per run): "
                    "hbm_bytes_per_launch = 128*TCC_EA0_RDREQ_128B + 64*TCC_EA0_RDREQ_64B + 32*TCC_EA0_RDREQ_32B + "
                    "WRITE_SIZE*1024 (L2-to-fabric bytes, Infinity Cache hits included; calibrated against known "
                    "bytes for 16-B vector, 48-B record and 64-B scalar reads and 4-/16-B stores, tools/calib); "
                    "FETCH_SIZE*2 (the x2 gfx950 correction, exact only for vector reads) kept as "
                    "fetch_x2_bytes_per_launch.  SQ_INSTS_VALU = VALU wave-instructions.  src_sha256 = the product "
                    "sources the counters were collected on; bench.py drops the measured fields when the tree's "
                    "sources differ.")
    json.dump(out, open(out_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:])
