"""A/B of the lane-refill bounce kernel (RT_OPT_BOUNCE_REFILL) against the
one-pixel-per-lane kernel: device time per frame (HIP events around K
rt_render_async calls on one stream, interleaved repeats) and the images'
bits.  Prints one JSON line per config.

    python tools/refill_ab.py --configs c4s7 c4s9 c4 [--steps 10] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c4s7", "c4s9"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    import rt_amd

    for cfg in args.configs:
        name, W, H, depth = bench.CONFIGS[cfg]
        scene = rt_amd.Scene(bench.scene_path(name), W, H, depth)
        ctxs = [rt_amd.Context(0, bounce_refill=v) for v in (0, 1)]
        outs = []
        for c in ctxs:
            c.upload(scene)
            outs.append(torch.empty((H, W, 4), dtype=torch.uint8, device="cuda"))
        st = torch.cuda.current_stream()
        for c, o in zip(ctxs, outs):
            c.render_async(scene.frame, o.data_ptr(), 0, st.cuda_stream)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs[0], outs[1]))
        ms = [[], []]
        for _ in range(args.reps):
            for i, (c, o) in enumerate(zip(ctxs, outs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.steps):
                    c.render_async(scene.frame, o.data_ptr(), 0, st.cuda_stream)
                e1.record()
                torch.cuda.synchronize()
                ms[i].append(e0.elapsed_time(e1) / args.steps)
        for c in ctxs:
            c.close()
        best = [min(m) for m in ms]
        print(json.dumps({"config": cfg, "same_bits": same, "ms_lanes": round(best[0], 4),
                          "ms_refill": round(best[1], 4), "refill_vs_lanes": round(best[1] / best[0], 4),
                          "all_ms": [[round(x, 4) for x in m] for m in ms]}), flush=True)


if __name__ == "__main__":
    main()
