"""Per-section shader-clock breakdown of the trace kernel (diagnostic).

Builds with -DRT_PROF accumulate s_memtime deltas per wave into 8 sections
(0 set-up, 1 primary closest hit, 2 shading set-up + light vectors, 3 wave
cones + shadow culling, 4 exact shadow triangle tests, 5 translucent filter +
Lambert/Phong, 6 store/stats, 7 shadow plane tests; marks are scheduling
barriers, so the build is slower than the product) and wave-level event
counts (cluster batches, member batches, exact tests per wave);
this renders a config K times with such a build and prints each section's
share of the summed wave time.

    python tools/prof_sections.py ray-tracing-gpu_amd/lib/var/prof.so --config c2
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
sys.path.insert(0, REPO)

# wave-level events (per wave): cluster batches, member batches, exact tests
EVENTS = ["cam_cluster_batches", "cam_member_batches", "cam_exact", "shadow_cluster_ballots",
          "shadow_member_batches", "shadow_exact", "shadow_clusters_by_dcap_only", "shadow_clusters_by_cone"]
# with the light buffer (shadow_opaque_lb), events 3-7 are its own
EVENTS_LB = ["lb_one_cell_walks", "lb_multi_cell_walks", EVENTS[2]] + ["lb_walk_iters", "lb_walk_exact", "lb_dcap_iters", "lb_fallback_waves", "lb_walk_active_lanes"]
NAMES = ["setup", "primary", "shade_setup", "shadow_cull", "shadow_exact_tri", "lambert_phong", "store", "shadow_planes"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="context option (rt_amd.OPTIONS), e.g. --option camera_buffer=0")
    a = ap.parse_args()
    opts = {k: float(v) for k, v in (o.split("=", 1) for o in a.option)}
    os.environ["RT_AMD_LIB"] = os.path.abspath(a.lib)
    import torch  # noqa: F401  (one HIP runtime)

    import bench
    import rt_amd

    L = rt_amd.lib()
    L.rt_debug_prof.argtypes = [ctypes.c_void_p]
    L.rt_debug_prof_events.argtypes = [ctypes.c_void_p]
    L.rt_debug_lb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    name, W, H, depth = bench.CONFIGS[a.config]
    s = rt_amd.Scene(bench.scene_path(name), W, H, depth)
    ctx = rt_amd.Context(0, **opts)
    ctx.upload(s)
    info = (ctypes.c_double * 30)()
    L.rt_debug_lb_info(ctx._h, info, 30)
    lbinfo = list(info)[: 3 + 3 * s.flat.n_lights] if info[0] else None
    ctx.render(s.frame)
    buf = (ctypes.c_ulonglong * 8)()
    ev = (ctypes.c_ulonglong * 8)()
    L.rt_debug_prof(buf)  # clear
    L.rt_debug_prof_events(ev)
    for _ in range(a.frames):
        ctx.render(s.frame)
    L.rt_debug_prof(buf)
    L.rt_debug_prof_events(ev)
    waves = ((W + 7) // 8) * ((H + 7) // 8) * a.frames
    ev_names = EVENTS_LB if lbinfo else EVENTS
    tot = sum(buf[:8]) or 1
    print(json.dumps({"config": a.config, "options": opts, "frames": a.frames,
                      "share": {n: round(buf[i] / tot, 4) for i, n in enumerate(NAMES)},
                      "wave_clocks_per_frame": {n: buf[i] // a.frames for i, n in enumerate(NAMES)},
                      "events_per_wave": {n: round(ev[i] / waves, 2) for i, n in enumerate(ev_names) if n},
                      "light_buffer": lbinfo}))


if __name__ == "__main__":
    main()
