"""Light 0's first light-buffer resolution R (6 R^2 cells) of a bench config's
scene, and the wavefront frame's bounce rays per level, from
rt_debug_upload_info out[9] and rt_debug_wf_counts.

    python tools/lb_res.py c3r c5r
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def main(configs):
    import bench
    import rt_amd

    L = rt_amd.lib()
    L.rt_debug_upload_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    for cfg in configs:
        name, W, H, depth = bench.CONFIGS[cfg]
        s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
        ctx = rt_amd.Context(0)
        ctx.upload(s)
        ctx.render_float(s.frame)
        out = (ctypes.c_double * 10)()
        assert L.rt_debug_upload_info(ctx._h, out, 10) == 0
        R = int(out[9])
        print(json.dumps({"config": cfg, "lb_R": R, "cells": 6 * R * R, "kernel": ctx.stats().kernel}))
        ctx.close()


if __name__ == "__main__":
    main(sys.argv[1:] or ["c3r"])
