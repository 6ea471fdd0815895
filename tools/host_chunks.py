"""Synchronous host-buffer renders (rt_render into pinned host memory) with
and without row chunks (RT_OPT_HOST_CHUNK_MB), static and moving camera.

    python tools/host_chunks.py --config c5
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def main():
    import ctypes

    import torch

    import bench
    import rt_amd

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--frames", type=int, default=8)
    a = ap.parse_args()
    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    L = rt_amd.lib()
    pin = torch.empty((H, W, 4), dtype=torch.uint8).pin_memory()
    out = {}
    for mb in (0, 64, 32, 16, 8):
        ctx = rt_amd.Context(0, host_chunk_mb=mb)
        ctx.upload(s)
        L.rt_render(ctx._h, ctypes.byref(s.frame), pin.data_ptr())
        t0 = time.perf_counter()
        for _ in range(a.frames):
            L.rt_render(ctx._h, ctypes.byref(s.frame), pin.data_ptr())
        static = (time.perf_counter() - t0) * 1e3 / a.frames
        path = rt_amd.camera_path(s.frame, a.frames + 1, yaw_deg=0.0, step=(0.37, 0.0, -0.21))
        L.rt_render(ctx._h, ctypes.byref(path[0]), pin.data_ptr())
        t0 = time.perf_counter()
        for f in path[1:]:
            L.rt_render(ctx._h, ctypes.byref(f), pin.data_ptr())
        moving = (time.perf_counter() - t0) * 1e3 / a.frames
        out[f"chunk_mb_{mb}"] = {"static_ms": round(static, 3), "moving_ms": round(moving, 3),
                                 "kernel_ms": round(ctx.stats().kernel_ms, 3)}
        ctx.close()
    print(json.dumps({"config": a.config, "pinned_host_render": out}))


if __name__ == "__main__":
    main()
