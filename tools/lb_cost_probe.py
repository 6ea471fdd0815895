import ctypes, json, sys, time
sys.path.insert(0, "ray-tracing-gpu_amd"); sys.path.insert(0, ".")
import torch, bench, rt_amd
L = rt_amd.lib()
L.rt_debug_lb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
name, W, H, d = bench.CONFIGS["c3"]
s = rt_amd.Scene(bench.scene_path(name), W, H, d)
for sc in (0, 6, 0, 6):
    ctx = rt_amd.Context(0, **({"lb_scale": sc} if sc else {}))
    t0 = time.perf_counter(); ctx.upload(s); t1 = time.perf_counter()
    info = (ctypes.c_double * 30)(); L.rt_debug_lb_info(ctx._h, info, 30)
    print(json.dumps({"lb_scale": sc, "upload_ms": round((t1 - t0) * 1e3, 1), "entries": info[1], "build_ms": round(info[2], 1), "R": [info[3], info[6]]}))
    del ctx
