"""A/B timing of librt_amd build variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Each variant .so is loaded with
RTLD_LOCAL so their identical symbol names do not collide.

    python tools/ab_variants.py --config c2 lib/var/librt_amd_base.so lib/var/librt_amd_nosl.so ...

A variant may carry context options (rt_set_option, names as in
rt_amd.OPTIONS) set before its upload, e.g. lib/librt_amd.so@lb_scale=2
(several: @a=1,b=2; the far light-buffer ladder as far=6:64).
--moving: each round renders a path of moved cameras (a new camera every
frame, as bench.py's moving-camera leg) instead of the static camera.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)


def load(path):
    import rt_amd

    L = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    for name, (res, args) in rt_amd.SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


def main():
    import torch

    import bench
    import rt_amd

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--moving", action="store_true")
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    name, W, H, depth = bench.CONFIGS[a.config]
    path = bench.scene_path(name)
    out = torch.zeros((H, W, 4), dtype=torch.uint8, device="cuda")
    ref = None
    vs = []
    for spec in a.libs:
        lp, _, envs = spec.partition("@")
        opts = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
        L = load(lp)
        sc = ctypes.c_void_p()
        assert L.rt_scene_create(ctypes.byref(sc)) == 0
        L.rt_scene_set_resolution(sc, W, H)
        L.rt_scene_set_max_bounces(sc, depth)
        assert L.rt_scene_load_file(sc, path.encode()) == 0
        assert L.rt_scene_prepare(sc) == 0
        flat, fr = rt_amd.SceneFlat(), rt_amd.Frame()
        L.rt_scene_get_flat(sc, ctypes.byref(flat))
        L.rt_scene_get_frame(sc, ctypes.byref(fr))
        ctx = ctypes.c_void_p()
        assert L.rt_create(0, ctypes.byref(ctx)) == 0
        for k, v in opts.items():
            if k == "far":
                fs = [float(x) for x in v.split(":") if x]
                arr = (ctypes.c_double * max(1, len(fs)))(*fs)
                assert L.rt_set_far_ladder(ctx, arr, len(fs)) == 0
            else:
                assert L.rt_set_option(ctx, rt_amd.OPTIONS[k], float(v)) == 0
        assert L.rt_upload_scene(ctx, ctypes.byref(flat)) == 0
        # one synchronous render first: it builds what is built per camera
        # (the camera buffer) exactly as bench.py's counted render does
        host = (ctypes.c_uint8 * (W * H * 4))()
        assert L.rt_render(ctx, ctypes.byref(fr), host) == 0
        L.rt_render_async(ctx, ctypes.byref(fr), out.data_ptr(), None, None)
        torch.cuda.synchronize()
        img = out.clone()
        same = True if ref is None else bool(torch.equal(img, ref))
        ref = img if ref is None else ref
        path_frames = []
        for k in range(a.frames):
            f = rt_amd.Frame()
            ctypes.pointer(f)[0] = fr
            f.cam_pos[0] -= 0.29 * (k + 1)
            f.cam_pos[2] += 0.17 * (k + 1)
            path_frames.append(f)
        vs.append(dict(lib=os.path.basename(lp) + ("@" + envs if envs else ""), L=L, ctx=ctx, fr=fr, sc=sc, times=[],
                       same_as_first=same, path=path_frames))
    for _ in range(a.rounds):
        for v in vs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(a.frames):
                f = v["path"][k] if a.moving else v["fr"]
                v["L"].rt_render_async(v["ctx"], ctypes.byref(f), out.data_ptr(), None, None)
            e1.record()
            torch.cuda.synchronize()
            v["times"].append(e0.elapsed_time(e1) / a.frames)
    res = [{"lib": v["lib"], "median_ms": round(statistics.median(v["times"]), 4),
            "min_ms": round(min(v["times"]), 4), "identical_output": v["same_as_first"]} for v in vs]
    print(json.dumps({"config": a.config, "moving": a.moving, "results": res}))


if __name__ == "__main__":
    main()
