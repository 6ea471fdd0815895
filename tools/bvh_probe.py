"""Where a reflective-heightfield frame's time goes (the BVH kernels,
rt_bvh.h): kernel time of the c3r scene (the 50k-triangle mesh with
`reflect: 0.5`) at 1920x1080 for max bounces 0..3 (0: the depth-0 kernel;
1..3: the BVH kernels), with the bounce-ray counters of an RT_FLAG_STATS
render beside each, and the plain mesh (c3) for comparison.

    python tools/bvh_probe.py [--frames 20] [--size 1920x1080] [--option NAME=VALUE ...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--depths", default="0,1,2,3")
    ap.add_argument("--option", action="append", default=[])
    a = ap.parse_args()
    import torch

    import rt_amd
    from rt_amd import synth

    W, H = map(int, a.size.split("x"))
    opts = {k: float(v) for k, v in (o.split("=", 1) for o in a.option)}
    paths = {"c3": synth.write_heightfield("/tmp/rt_amd_heightfield.dat"),
             "c3r": synth.write_heightfield("/tmp/rt_amd_heightfield_r05.dat", reflect=0.5)}
    out = {}
    stream = torch.cuda.current_stream().cuda_stream
    dev = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    for name, path in paths.items():
        ctx = rt_amd.Context(0, **opts)
        for d in map(int, a.depths.split(",")):
            if name == "c3" and d > 0:
                continue
            s = rt_amd.Scene(path, W, H, d)
            if d == int(a.depths.split(",")[0]) or name == "c3":
                ctx.upload(s)
            f = s.frame.copy()
            f.flags = rt_amd.FLAG_STATS
            ctx.render(f)
            st = ctx.stats()
            for _ in range(3):
                ctx.render_async(s.frame, dev.data_ptr(), 0, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.frames):
                ctx.render_async(s.frame, dev.data_ptr(), 0, stream)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.frames
            out[f"{name}_d{d}"] = {
                "ms": round(ms, 4), "kernel": ctx.stats().kernel, "bounce_rays": st.bounce_rays,
                "shadow_rays": st.shadow_rays,
                "bounce_tests_per_ray": round(st.bounce_triangle_tests / max(1, st.bounce_rays), 2),
                "bvh_nodes_per_ray": round(st.bvh_nodes_visited / max(1, st.bounce_rays), 2)}
            print(name, d, out[f"{name}_d{d}"], flush=True)
        ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
