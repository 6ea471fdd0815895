"""Per-tile cost map of the trace kernel (diagnostic, RT_PROF build).

Renders a config with a -DRT_PROF build of librt_amd.so and saves, per 8x8
tile, the wave's shader clocks (total and per section) and its event counts
(tools/prof_sections.py names them) to an .npz, then prints the tail: how
much of the summed wave time the most expensive tiles hold and which events
they ran.

    python tools/prof_tiles.py ray-tracing-gpu_amd/lib/var/prof.so --config c3 --out gpurun_out/tiles_c3.npz
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)
EV = ["cam_member_batches", "cam_exact", "shadow_member_batches", "shadow_exact", "shadow_clusters_by_dcap_only",
      "shadow_clusters_by_cone"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ["RT_AMD_LIB"] = os.path.abspath(a.lib)
    import numpy as np
    import torch

    import bench
    import rt_amd

    L = rt_amd.lib()
    L.rt_debug_prof_tiles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    ctx = rt_amd.Context(0)
    ctx.upload(s)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tw, th = 2 * gx, 2 * gy
    buf = torch.zeros((th * tw * 16,), dtype=torch.int32, device="cuda")
    assert L.rt_debug_prof_tiles(buf.data_ptr(), th * tw) == 0
    ctx.render(s.frame)
    torch.cuda.synchronize()
    assert L.rt_debug_prof_tiles(None, 0) == 0
    t = buf.view(th, tw, 16).cpu().numpy().view(np.uint32).astype(np.uint64)
    tot = t[..., 0] + (t[..., 1] << np.uint64(32))
    valid = np.zeros((th, tw), bool)
    valid[: (H + 7) // 8, : (W + 7) // 8] = True
    tv = tot[valid].astype(np.float64)
    order = np.sort(tv)[::-1]
    csum = np.cumsum(order) / order.sum()
    res = {"config": a.config, "tiles": int(valid.sum()), "mean_clk": float(tv.mean()), "max_clk": float(tv.max()),
           "p50_clk": float(np.median(tv)), "p99_clk": float(np.percentile(tv, 99)),
           "share_top1pct": float(csum[max(0, len(csum) // 100 - 1)]),
           "share_top10pct": float(csum[max(0, len(csum) // 10 - 1)])}
    top = np.argsort(tot * valid, axis=None)[::-1][:10]
    res["top_tiles"] = [{"row": int(i // tw), "col": int(i % tw), "clk": int(tot.flat[i]),
                         "events": {n: int(t.reshape(-1, 16)[i, 10 + k]) for k, n in enumerate(EV)}} for i in top]
    rows = (tot * valid).sum(axis=1).astype(np.float64)
    res["row_band_share"] = [round(float(x), 4) for x in np.add.reduceat(rows, np.arange(0, th, max(1, th // 16))) / rows.sum()]
    if a.out:
        np.savez_compressed(a.out, tot=tot, sec=t[..., 2:10], ev=t[..., 10:16], valid=valid)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
