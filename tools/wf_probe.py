"""Per-level picture of a wavefront frame (c3r / c5r): the queue counts of
each bounce level (rays, parents, straggling walks: rt_debug_wf_counts) and
N async frames for a kernel trace (tools/trace_seq.py splits it per launch).

    python tools/wf_probe.py --config c3r [--frames 20] [--option name=value]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3r")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--option", action="append", default=[])
    a = ap.parse_args()
    import torch

    import bench
    import rt_amd

    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    opts = {k: float(v) for k, v in (o.split("=", 1) for o in a.option)}
    c = rt_amd.Context(0, **opts)
    c.upload(s)
    out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        c.render_async(s.frame, out.data_ptr(), 0, st)
    torch.cuda.synchronize()
    L = rt_amd.lib()
    L.rt_debug_wf_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_uint * 27)()
    assert L.rt_debug_wf_counts(c._h, buf, 27) == 0, c._err()
    levels = [{"level": l, "rays": buf[3 * l], "parents": buf[3 * l + 1], "stragglers": buf[3 * l + 2]}
              for l in range(depth + 1)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.frames):
        c.render_async(s.frame, out.data_ptr(), 0, st)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"config": a.config, "options": opts, "levels": levels, "kernel": c.stats().kernel,
                      "ms_per_frame": round(e0.elapsed_time(e1) / a.frames, 4)}), flush=True)


if __name__ == "__main__":
    main()
