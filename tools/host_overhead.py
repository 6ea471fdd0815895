"""Host cost of one rt_render_async call (frozen camera, device output): the
enqueue rate bounds the frame rate of small frames.  Prints host us per call
over N calls without syncs, and device ms per frame over the same calls.

    python tools/host_overhead.py --config c1 [--n 2000]
"""
import argparse
import ctypes
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
    ap.add_argument("--config", default="c1")
    ap.add_argument("--n", type=int, default=2000)
    a = ap.parse_args()
    import torch

    import rt_amd

    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    ctx.render(s.frame)
    dev = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    L = rt_amd.lib()
    fr = ctypes.byref(s.frame)
    ptr = ctypes.c_void_p(dev.data_ptr())
    h = ctx._h
    for _ in range(200):
        L.rt_render_async(h, fr, ptr, None, ctypes.c_void_p(st))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for _ in range(a.n):
        L.rt_render_async(h, fr, ptr, None, ctypes.c_void_p(st))
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"config": a.config, "host_us_per_call": round((t1 - t0) * 1e6 / a.n, 2),
                      "device_ms_per_frame": round(e0.elapsed_time(e1) / a.n, 4)}))
    ctx.close()


if __name__ == "__main__":
    main()
