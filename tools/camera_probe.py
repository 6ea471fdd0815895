"""Per-camera cost probe: renders a moving camera (translated every frame)
through the synchronous path (camera prepass + camera buffer + kernel), the
async path and the sequence path, so that `rocprofv3 --kernel-trace --stats
-- python tools/camera_probe.py --config c3` shows each per-camera kernel's
device time.  Prints one JSON line of host-side per-frame times.

    python tools/camera_probe.py --config c3 [--frames 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--cb", type=int, default=1, help="RT_OPT_CAMERA_BUFFER")
    args = ap.parse_args()
    import torch

    import rt_amd

    name, W, H, depth = bench.CONFIGS[args.config]
    scene = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    ctx = rt_amd.Context(0, camera_buffer=args.cb)
    ctx.upload(scene)
    dev = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    n = args.frames

    def cams(sx, sz):
        out = []
        for k in range(n + 1):
            f = scene.frame.copy()
            f.cam_pos[0] += sx * (k + 1)
            f.cam_pos[2] += sz * (k + 1)
            out.append(f)
        return out

    res = {"config": args.config, "cb": args.cb}
    fr = cams(0.37, -0.21)
    ctx.render_async(scene.frame, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    # static camera, async
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.render_async(scene.frame, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    res["static_async_ms"] = round((time.perf_counter() - t0) * 1e3 / n, 4)
    # moving camera, synchronous into device memory
    ctx.prepare_camera(fr[0])
    t0 = time.perf_counter()
    for f in fr[1:]:
        ctx.prepare_camera(f)
        ctx.render_async(f, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    res["moving_prepare_then_async_ms"] = round((time.perf_counter() - t0) * 1e3 / n, 4)
    fr = cams(-0.29, 0.17)
    ctx.render_async(fr[0], dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in fr[1:]:
        ctx.render_async(f, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    res["moving_async_ms"] = round((time.perf_counter() - t0) * 1e3 / n, 4)
    res["same_cameras"] = bench.moving_camera_events(ctx, fr[1:], dev.data_ptr(), stream)
    ring = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    path = rt_amd.camera_path(scene.frame, n, yaw_deg=0.25, step=(0.3, 0.0, -0.2))
    ctx.render_sequence_async(path, ring.data_ptr(), H * W * 4, 0, 0, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.render_sequence_async(path, ring.data_ptr(), H * W * 4, 0, 0, stream)
    torch.cuda.synchronize()
    res["sequence_ms"] = round((time.perf_counter() - t0) * 1e3 / n, 4)
    import ctypes

    L = rt_amd.lib()
    L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    ci = (ctypes.c_double * 10)()
    ctx.prepare_camera(scene.frame)
    if L.rt_debug_cb_info(ctx._h, ci, 10) == 0:
        res["cbinfo"] = {"valid": ci[0], "entries": ci[1], "build_ms": round(ci[2], 4), "candidate_pairs": ci[6],
                     "lists_over_256": ci[7], "longest": ci[8], "capacity": ci[9]}
    ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
