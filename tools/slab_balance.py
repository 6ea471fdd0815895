"""Load balance of row-slab sharding (diagnostic, one GPU).

Renders each rank's slab of a config on its own, for n = 2, 4, 8 ranks, and
reports the slab kernel times: the multi-GPU step can be no faster than the
slowest slab (bands instead of slabs past ~10% imbalance).

    python tools/slab_balance.py --config c2 c3 c5
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def time_frame(ctx, fr, out, stream, frames):
    """Kernel ms of fr's share, its camera prepared first (the camera buffer
    for its rows: the kernel bench.py's ranks time)."""
    import torch

    ctx.prepare_camera(fr)
    ctx.render_async(fr, out.data_ptr(), 0, stream)
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(frames):
            ctx.render_async(fr, out.data_ptr(), 0, stream)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / frames)
    return statistics.median(ts)


def main():
    import torch

    import bench
    import rt_amd
    from rt_amd.dist import slab_rows

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", nargs="+", default=["c2"])
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--bands", type=int, default=0, help="also time cyclic bands of this many rows")
    a = ap.parse_args()
    stream = torch.cuda.current_stream().cuda_stream
    res = {}
    for cfg in a.config:
        name, W, H, depth = bench.CONFIGS[cfg]
        s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
        ctx = rt_amd.Context(0)
        ctx.upload(s)
        out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
        frames = a.frames if W * H <= 4_000_000 else max(2, a.frames // 4)
        t0 = time.perf_counter()  # clock settle (bench.py --settle-ms)
        while time.perf_counter() - t0 < 0.3:
            time_frame(ctx, s.frame, out, stream, 2)
        full = time_frame(ctx, s.frame, out, stream, frames)
        r = {"full_ms": round(full, 4)}
        for n in (2, 4, 8):
            ts = []
            for rank in range(n):
                r0, r1, _ = slab_rows(H, n, rank)
                fr = s.frame.copy()
                fr.row_begin, fr.row_end = r0, r1
                ts.append(time_frame(ctx, fr, out, stream, frames))
            bs = []
            for rank in range(n):  # cyclic 16-row bands (rt_frame.band_rows)
                fr = s.frame.copy()
                fr.band_rows, fr.band_count, fr.band_index = 16, n, rank
                bs.append(time_frame(ctx, fr, out, stream, frames))
            r[f"n{n}"] = {"slab_ms": [round(t, 4) for t in ts], "max_ms": round(max(ts), 4),
                          "imbalance": round(max(ts) / (sum(ts) / n) - 1.0, 3),
                          "ideal_speedup": round(full / max(ts), 2),
                          "band_ms": [round(t, 4) for t in bs], "band_imbalance": round(max(bs) / (sum(bs) / n) - 1.0, 3),
                          "band_ideal_speedup": round(full / max(bs), 2)}
        res[cfg] = r
        print(json.dumps({cfg: r}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
