"""Upload-time breakdown of the light-buffer build (diagnostic): uploads a
config's scene into fresh contexts and prints rt_debug_upload_info's parts
(copy + records, prepasses, light buffer, total) and the light buffer's
phases (cone records to the host, host preparation, supercell counts,
supercell lists + cell counts, entries).

    python tools/lb_phases.py --config c3 --reps 3
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401

    import bench
    import rt_amd

    L = rt_amd.lib()
    fn = L.rt_debug_upload_info
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    names = ["records_and_copies", "prepasses", "light_buffer", "total", "cones_to_host", "host_prep",
             "supercell_counts", "supercell_lists_cell_counts", "entries"]
    for r in range(a.reps):
        ctx = rt_amd.Context(0)
        t0 = time.perf_counter()
        ctx.upload(s)
        t1 = time.perf_counter()
        buf = (ctypes.c_double * 9)()
        fn(ctx._h, buf, 9)
        print(json.dumps({"rep": r, "upload_wall_ms": round((t1 - t0) * 1e3, 2),
                          **{n: round(buf[i], 2) for i, n in enumerate(names)}}))
        del ctx


if __name__ == "__main__":
    main()
