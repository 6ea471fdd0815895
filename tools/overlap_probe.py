"""Frames in flight (diagnostic): ms/frame of rt_render_async with one
stream against S streams round-robin (separate output buffers, so frame
k+1's kernel may overlap frame k's), for the full frame and for one rank's
1/n row slab (the N>1 per-rank work).

    python tools/overlap_probe.py --config c2
"""
import argparse
import copy
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    import torch

    import bench
    import rt_amd
    from rt_amd.dist import slab_rows

    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    streams = [torch.cuda.Stream() for _ in range(4)]
    out = []
    for n in (1, 2, 4, 8):
        r0, r1, rows = slab_rows(H, n, n // 2)  # a middle slab (mesh rows for the heightfield)
        f = copy.copy(s.frame)
        f.row_begin, f.row_end = r0, r1
        bufs = [torch.zeros((rows, W, 4), dtype=torch.uint8, device="cuda") for _ in range(4)]
        ctx.render(f)  # camera buffer for these rows
        res = {"slab_of": n, "rows": r1 - r0}
        for S in (1, 2, 3, 4):
            for rep in range(2):  # second rep is the measurement (settled clock)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                cur = torch.cuda.current_stream()
                e0.record(cur)
                for st in streams[:S]:
                    st.wait_stream(cur)
                for k in range(a.frames):
                    st = streams[k % S]
                    ctx.render_async(f, bufs[k % S].data_ptr(), 0, st.cuda_stream)
                for st in streams[:S]:
                    cur.wait_stream(st)
                e1.record(cur)
                torch.cuda.synchronize()
            res[f"streams{S}_ms_per_frame"] = round(e0.elapsed_time(e1) / a.frames, 4)
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
