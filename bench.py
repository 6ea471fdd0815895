"""bench.py — the reference's headline metric on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

Metric (BASELINE.json): Mray/s and ms/frame at 1920x1080 depth=3 on 1/2/4/8
MI355X vs host CPU.  A step renders ONE full frame of the configured workload
(default C2 = the reference's scene2.dat at 1920x1080, max bounces 3) from a
scene already resident in HBM into an RGBA8 framebuffer in HBM.  With N ranks
(one process per GPU, torch.distributed over RCCL) every rank renders its
contiguous row slab and the slabs are gathered to rank 0 with grouped RCCL
point-to-point transfers over xGMI (rt_amd.dist.RootGather, double-buffered so
frame k's gather overlaps frame k+1's render); the timed region ends after the
last gather (strong scaling: the frame is fixed).

value = primary rays (= pixels) of all ranks / max-over-ranks time, in Mray/s.
The roofline entry prices the trace kernel against the FP32 vector peak with
the reference algorithm's operation count; the CPU baseline
times the reference's own primitive code (oracle/_ref) on host cores over a
bounded sample of the same frame.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ray-tracing-gpu_amd"))
SCENES = os.path.join(REPO, "tests", "golden", "scenes")

# FP32 operations per work item of the reference algorithm.
OPS_TRI, OPS_PLANE, OPS_QUAD = 52, 12, 103
OPS_RAY_SETUP, OPS_SHADE_PER_LIT_LIGHT = 34, 75
PEAK_FP32_TFLOPS = 157.3          # MI355X_MICROARCH.md: FP32 vector (= dense f32 MFMA) peak
PEAK_NOFMA_TOPS = 78.6            # no FMA allowed by parity: packed v_pk_mul/add, 1 op/lane/clk x2

CONFIGS = {
    "c1": ("scene1.dat", 512, 512, 1),
    "c2": ("scene2.dat", 1920, 1080, 3),
    "c3": ("heightfield", 1920, 1080, 1),
    "c4": ("scene2.dat", 3840, 2160, 5),
    "c4s7": ("scene7.dat", 3840, 2160, 5),
    "c4s9": ("scene9.dat", 3840, 2160, 5),
    "c5": ("heightfield", 7680, 4320, 3),
    # SURVEY 8(d) C5's "--reflect 0.5" variant: every triangle a mirror, so
    # every bounce ray walks the 50k-triangle mesh (the BVH kernels)
    "c3r": ("heightfield_r05", 1920, 1080, 3),
    "c5r": ("heightfield_r05", 7680, 4320, 3),
}


def product_src_sha256() -> str:
    """Hash of the product's kernel sources and build flags (the code the PMC
    counters in profiles/pmc.json were collected on)."""
    import hashlib

    h = hashlib.sha256()
    pkg = os.path.join(REPO, "ray-tracing-gpu_amd")
    for rel in sorted(os.listdir(os.path.join(pkg, "csrc"))):
        with open(os.path.join(pkg, "csrc", rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    for path in (os.path.join(pkg, "Makefile"), os.path.join(REPO, "include", "rt.h")):
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def scene_path(name: str) -> str:
    if name.startswith("heightfield"):
        from rt_amd import synth

        if name == "heightfield_r05":
            return synth.write_heightfield(os.path.join("/tmp", "rt_amd_heightfield_r05.dat"), reflect=0.5)
        return synth.write_heightfield(os.path.join("/tmp", "rt_amd_heightfield.dat"))
    return os.path.join(SCENES, name)


def algorithmic_flops(types, primary, bounce, shadow):
    """The reference algorithm's volume: every ray against every surface."""
    import numpy as np

    per_ray = (int(np.sum(types == 0)) * OPS_TRI + int(np.sum(types == 1)) * OPS_PLANE +
               int(np.sum(types == 2)) * OPS_QUAD)
    return (primary + bounce + shadow) * per_ray + primary * OPS_RAY_SETUP + shadow * OPS_SHADE_PER_LIT_LIGHT


def executed_flops(st):
    """tests the kernel actually executed (rt_stats, a wave-level
    test counted once per lane of the wave) x ops per test, plus ray set-up and
    shading per lit light."""
    return (st.triangle_tests * OPS_TRI + st.plane_tests * OPS_PLANE + st.quadric_tests * OPS_QUAD +
            st.primary_rays * OPS_RAY_SETUP + st.shadow_rays * OPS_SHADE_PER_LIT_LIGHT)


def cpu_baseline(path, w, h, depth, seconds):
    """Time the reference's own primitive code (oracle/_ref, serial like the
    reference) on 8x8 windows spread over the frame until `seconds` elapse;
    fall back to the C restatement (oracle/liboracle.so) when _ref was not built."""
    import numpy as np

    ref = os.path.join(REPO, "oracle", "_ref", "libref_oracle.so")
    port = os.path.join(REPO, "oracle", "liboracle.so")
    VP = ctypes.c_void_p
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        kind, load, rend, free = "reference", L.ref_load, L.ref_render_window, L.ref_free
        rend.argtypes = [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP]
        call = lambda p, r0, r1, c0, c1, buf: rend(p, r0, r1, c0, c1, buf)
    else:
        if not os.path.exists(port):
            import subprocess

            subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
        L = ctypes.CDLL(port)
        kind, load, rend, free = "port", L.oracle_load, L.oracle_render_window, L.oracle_free
        rend.argtypes = [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, ctypes.c_int]
        call = lambda p, r0, r1, c0, c1, buf: rend(p, r0, r1, c0, c1, buf, 1)
    load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(VP)]
    free.argtypes = [VP]
    p = VP()
    assert load(path.encode(), w, h, depth, ctypes.byref(p)) == 0
    buf = np.zeros((8, 8, 3), np.float32)
    # 8x8 windows on a coarse grid, visited in a fixed scrambled order
    wins = [(r, c) for r in range(0, h - 7, max(8, h // 32)) for c in range(0, w - 7, max(8, w // 32))]
    order = np.random.default_rng(1234).permutation(len(wins))
    px = 0
    t0 = time.perf_counter()
    k = 0
    while True:
        r, c = wins[order[k % len(wins)]]
        call(p, r, r + 8, c, c + 8, buf.ctypes.data)
        px += 64
        k += 1
        el = time.perf_counter() - t0
        if el >= seconds and k >= min(len(wins), 64):
            break
    free(p)
    return {"value": round(px / el / 1e6, 4), "unit": "Mray/s", "cores": 1, "kind": kind,
            "sample": f"{k} 8x8 windows ({px} primary rays) on a {len(wins)}-window grid over the "
                      f"{w}x{h} depth={depth} frame, {el:.1f} s, serial like the reference loop"}


def cpu_allcores(path, w, h, depth, seconds):
    """the C restatement (oracle/liboracle.so, OpenMP over
    rows, bit-identical to the reference) on all the host cores this job may
    use, over 64x64 windows spread over the frame until `seconds` elapse."""
    import numpy as np

    port = os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(port):
        import subprocess

        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    L = ctypes.CDLL(port)
    VP = ctypes.c_void_p
    L.oracle_load.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(VP)]
    L.oracle_render_window.argtypes = [VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, VP, ctypes.c_int]
    L.oracle_free.argtypes = [VP]
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)), os.cpu_count() or 1))
    p = VP()
    assert L.oracle_load(path.encode(), w, h, depth, ctypes.byref(p)) == 0
    n = 64
    buf = np.zeros((n, n, 3), np.float32)
    wins = [(r, c) for r in range(0, max(1, h - n + 1), max(n, h // 8)) for c in range(0, max(1, w - n + 1), max(n, w // 8))]
    order = np.random.default_rng(4321).permutation(len(wins))
    px, k = 0, 0
    t0 = time.perf_counter()
    while True:
        r, c = wins[order[k % len(wins)]]
        L.oracle_render_window(p, r, min(h, r + n), c, min(w, c + n), buf.ctypes.data, threads)
        px += (min(h, r + n) - r) * (min(w, c + n) - c)
        k += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    L.oracle_free(p)
    return {"value": round(px / el / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{k} 64x64 windows ({px} primary rays) of the {w}x{h} depth={depth} frame, "
                      f"{el:.1f} s, OpenMP over rows"}


def host_boundary(ctx, frame, W):
    """The drop-in's host-buffer form (not `value`): synchronous rt_render into
    host memory, as the reference's CScene::LancerRayons hands its frame to
    glTexImage2D from host memory (Scene.cpp:1562) — the kernel, the RGBA8
    device-to-host copy over PCIe and the host sync, per frame, into a
    pageable (numpy) and a pinned (torch) buffer."""
    import numpy as np
    import torch

    import rt_amd

    L = rt_amd.lib()
    rows = rt_amd.frame_rows(frame)
    frames = 20 if W * rows <= 4_000_000 else 5
    page = np.empty((rows, W, 4), np.uint8)
    pinned = torch.empty((rows, W, 4), dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    res = {}
    for kind, ptr in (("pageable", page.ctypes.data), ("pinned", pinned.data_ptr())):
        if L.rt_render(ctx._h, ctypes.byref(frame), ptr) != 0:
            return {"error": (L.rt_last_error(ctx._h) or b"").decode()}
        t0 = time.perf_counter()
        for _ in range(frames):
            L.rt_render(ctx._h, ctypes.byref(frame), ptr)
        ms = (time.perf_counter() - t0) * 1e3 / frames
        res[kind] = {"ms_per_frame": round(ms, 4), "mray_s": round(W * rows / ms / 1e3, 1)}
    res["bytes_per_frame"] = int(W * rows * 4)
    res["frames"] = frames
    res["note"] = ("rt_render (synchronous) into host memory: kernel + RGBA8 device-to-host copy over PCIe + "
                   "host sync; the PCIe-inclusive rate, never `value`")
    return res


def _debug(L, name, ctx, n):
    """rt_debug_* summaries (diagnostic exports, not in rt.h) as a list."""
    if not hasattr(L, name):
        return None
    fn = getattr(L, name)
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_double * n)()
    return list(buf) if fn(ctx._h, buf, n) == 0 else None


def progressive(ctx, frame, W, rows, n=60):
    """SURVEY 8(f) row 4, the headless analogue of the reference's GLUT
    display loop (Main.cpp:229-250): a camera path of n frames (yaw + move
    per frame) rendered on the device into a ring of RGBA8 frames in HBM with
    rt_render_sequence_async — enqueued directly, and captured once into a
    hipGraph and replayed.  Frames per second of the whole path."""
    import torch

    import rt_amd

    path = rt_amd.camera_path(frame, n, yaw_deg=0.25, step=(0.3, 0.0, -0.2))
    ring = torch.empty((n, rows, W, 4), dtype=torch.uint8, device="cuda")
    stride = rows * W * 4
    stream = torch.cuda.current_stream().cuda_stream
    ctx.render_sequence_async(path, ring.data_ptr(), stride, 0, 0, stream)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ctx.render_sequence_async(path, ring.data_ptr(), stride, 0, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    direct = (time.perf_counter() - t0) / (3 * n)
    import gc

    g = torch.cuda.CUDAGraph()
    gc.collect()
    gc.disable()  # no finalizer may synchronise a stream during the capture
    try:
        with torch.cuda.graph(g):
            ctx.render_sequence_async(path, ring.data_ptr(), stride, 0, 0, torch.cuda.current_stream().cuda_stream)
    finally:
        gc.enable()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / (3 * n)
    return {"frames": n, "stream_fps": round(1.0 / direct, 1), "graph_fps": round(1.0 / graph, 1),
            "graph_ms_per_frame": round(graph * 1e3, 4),
            "note": "camera path (0.25 deg yaw + move per frame) rendered into an HBM ring by "
                    "rt_render_sequence_async: per frame the camera prepasses, the slot's camera buffer where its "
                    "build pays (big lists, >= 4 Mpx) and the trace kernel; enqueued directly vs one hipGraph "
                    "replay per path"}


def frame_costs(scene, frame, W, cold, opts=None):
    """What the drop-in pays beyond the steady-state kernel (never `value`):
    the reference renders ONE frame per process through LancerRayons
    (Main.cpp:181, Scene.cpp:672), paying the scene upload, the per-camera
    structures and the kernel together.

    * first_frame_ms: a fresh context in a warm process — rt_upload_scene
      (device copy, cone / cluster prepasses, light buffer) + the first
      synchronous rt_render into pinned host memory (camera prepass, camera
      buffer, kernel, RGBA8 copy over PCIe);
    * cold: the same for the process's first context (adds the runtime's
      one-time code-object load), measured by main() before anything else;
    * moving camera: the camera translated every frame — synchronous
      rt_render into pinned host memory (prepass + camera buffer + kernel +
      copy), and rt_render_async into device memory (prepass, and the
      camera buffer where its build pays, on the stream), per frame."""
    import torch

    import rt_amd

    L = rt_amd.lib()
    rows = rt_amd.frame_rows(frame)
    pinned = torch.empty((rows, W, 4), dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    ctx = rt_amd.Context(0, **(opts or {}))
    t0 = time.perf_counter()
    ctx.upload(scene)
    t1 = time.perf_counter()
    if L.rt_render(ctx._h, ctypes.byref(frame), pinned.data_ptr()) != 0:
        return {"error": ctx._err()}
    t2 = time.perf_counter()
    up = _debug(L, "rt_debug_upload_info", ctx, 9)
    cb = _debug(L, "rt_debug_cb_info", ctx, 6)
    res = {"first_frame_ms": round((t2 - t0) * 1e3, 3), "upload_ms": round((t1 - t0) * 1e3, 3),
           "first_render_ms": round((t2 - t1) * 1e3, 3),
           "upload_parts_ms": {"records_and_copies": round(up[0], 3), "prepasses": round(up[1], 3),
                               "light_buffer": round(up[2], 3),
                               "light_buffer_phases": {"cones_to_host": round(up[4], 3), "host_prep": round(up[5], 3),
                                                       "supercell_counts": round(up[6], 3),
                                                       "supercell_lists_cell_counts": round(up[7], 3),
                                                       "entries": round(up[8], 3)}} if up else None,
           "camera_buffer_build_ms": round(cb[2], 3) if cb else None, "cold": cold}
    nfr = 20 if W * rows <= 4_000_000 else 8
    frames = []
    for k in range(nfr + 1):
        f = frame.copy()
        f.cam_pos[0] += 0.37 * (k + 1)
        f.cam_pos[2] -= 0.21 * (k + 1)
        frames.append(f)
    L.rt_render(ctx._h, ctypes.byref(frames[0]), pinned.data_ptr())
    t0 = time.perf_counter()
    for f in frames[1:]:
        L.rt_render(ctx._h, ctypes.byref(f), pinned.data_ptr())
    sync_ms = (time.perf_counter() - t0) * 1e3 / nfr
    dev = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    frames2 = []
    for k in range(nfr + 1):
        f = frame.copy()
        f.cam_pos[0] -= 0.29 * (k + 1)
        f.cam_pos[2] += 0.17 * (k + 1)
        frames2.append(f)
    ctx.render_async(frames2[0], dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in frames2[1:]:
        ctx.render_async(f, dev.data_ptr(), 0, stream)
    torch.cuda.synchronize()
    async_ms = (time.perf_counter() - t0) * 1e3 / nfr
    ev = moving_camera_events(ctx, frames2[1:], dev.data_ptr(), stream)
    res["moving_camera_ms_per_frame"] = round(sync_ms, 4)
    res["progressive"] = progressive(ctx, frame, W, rows)
    res["moving_camera"] = {"sync_host_ms_per_frame": round(sync_ms, 4),
                            "async_device_ms_per_frame": round(async_ms, 4), "frames": nfr,
                            "same_cameras": ev,
                            "note": "camera translated every frame; sync = rt_render into pinned host memory "
                                    "(camera prepass + camera buffer + kernel + PCIe copy); async = "
                                    "rt_render_async into HBM, no host sync: the camera prepass, and the camera "
                                    "buffer where its build pays (big lists, >= 4 Mpx), on the stream"}
    ctx.close()
    return res


def moving_camera_events(ctx, frames, dst, stream, repeats=3):
    """The per-camera cost, apart from the picture: each moved camera rendered
    1 + `repeats` times in a row, one HIP event pair around each launch on the
    render stream — the camera's first frame (its per-camera work: prepasses,
    camera buffer or tile masks) against the same camera's later frames (a
    static camera at that position).  A moved camera sees a different picture
    than the bench's static one, so only this pair isolates the per-camera cost."""
    import torch

    assert stream == torch.cuda.current_stream().cuda_stream  # the events' stream
    first, again = [], []
    for f in frames:
        for r in range(1 + repeats):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.render_async(f, dst, 0, stream)
            e1.record()
            (first if r == 0 else again).append((e0, e1))
    torch.cuda.synchronize()
    a = sorted(e0.elapsed_time(e1) for e0, e1 in first)
    b = sorted(e0.elapsed_time(e1) for e0, e1 in again)
    na, nb = a[len(a) // 2], b[len(b) // 2]
    return {"new_camera_ms": round(na, 4), "same_camera_ms": round(nb, 4), "ratio": round(na / nb, 3),
            "cameras": len(frames), "repeats": repeats,
            "note": "medians of per-launch HIP event pairs (dispatch gap included) over the moved cameras: each "
                    "camera's first frame vs the same camera's next frames"}


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` run bare: start the N ranks (one process per GPU)
    with torch.distributed.run as a child process — never an exec: this
    process has not touched the GPU and stays the parent — on a free local
    port, the same arguments forwarded; rank 0's JSON line goes straight to
    our stdout.  Returns the launcher's exit code."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")  # the launcher's default; silences its warning
    rc = subprocess.run(cmd, env=env).returncode
    if rc != 0:
        # a rank failed (its own message is above): the launcher stopped the
        # others, or they failed at their collective deadline
        print(f"bench.py: the {n}-rank run exited with status {rc}", file=sys.stderr, flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed renders for this long before the warmup steps, so the timed steps run at the "
                         "GPU's sustained clock (runs of a few dozen frames measured 6-9%% slower)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-boundary", action="store_true",
                    help="skip the PCIe-inclusive rt_render leg (profiling runs: only the timed launches)")
    ap.add_argument("--partition", default="auto", choices=["auto", "slabs", "bands"],
                    help="N>1: row slabs, cyclic 16-row bands, or bands when slabs are >10%% imbalanced")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 collective backend: nccl (= RCCL over xGMI, the benchmark) or gloo (the "
                         "gather staged through host memory; lets several ranks share one GPU for tests)")
    ap.add_argument("--gather-batch", type=int, default=4,
                    help="N>1: frames per gather collective (RCCL's fixed cost per call is comparable to a 1/N "
                         "slab of a 1080p frame; 1 = one gather per frame)")
    ap.add_argument("--gather-channels", type=int, default=3, choices=[3, 4],
                    help="N>1: bytes per pixel the gather carries (3: RGB, rank 0 restores the RGBA8 frame's "
                         "constant alpha; 4: the RGBA8 pixels as rendered)")
    ap.add_argument("--force-dist", action="store_true",
                    help="create the process group and run the gather path even with WORLD_SIZE=1 (exercises "
                         "RCCL's init, all-reduce and gather on a 1-GPU box)")
    ap.add_argument("--rank-timeout", type=float, default=180.0,
                    help="N>1: seconds any rank waits at the rendezvous or in a collective for a peer before it "
                         "fails (a dead or hung rank ends the run with a message instead of holding the node)")
    ap.add_argument("--frame-sha", action="store_true",
                    help="rank 0 adds the SHA-256 of the last assembled RGBA8 frame (bottom row first)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="context option (rt_amd.OPTIONS) for an A/B run, e.g. --option camera_buffer=2; "
                         "none changes an image")
    args = ap.parse_args()
    ctx_opts = {k: float(v) for k, v in (o.split("=", 1) for o in args.option)}

    # --gpus N is the number of ranks.  Launched bare (no WORLD_SIZE), N > 1
    # starts N ranks itself — torch.distributed.run as a CHILD process, before
    # this process touches torch or the GPU — and exits with its code (rank 0
    # prints the JSON line).  Under a launcher the world must be N.
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: refusing to report "
              f"{os.environ['WORLD_SIZE']} rank(s) as {args.gpus} GPU(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    if world > 1 and args.dist_backend == "nccl" and world > torch.cuda.device_count():
        # RCCL needs one GPU per rank ("Duplicate GPU detected"); gloo ranks may share one
        print(f"bench.py: {world} RCCL ranks but {torch.cuda.device_count()} visible GPU(s); use "
              f"--dist-backend gloo to share GPUs", file=sys.stderr, flush=True)
        sys.exit(2)

    from rt_amd.dist import rank_guard

    with rank_guard(rank):
        run_rank(args, ctx_opts, world, rank, local)


def dist_setup(backend: str, device: int, world: int, timeout_s: float):
    """The process group (RCCL, or gloo), with a deadline on the rendezvous and
    on every collective (rt_amd.dist.init_ranks), and the check that every
    rank joined: returns (dist, ranks_seen, gpus_used)."""
    import torch
    import torch.distributed as dist

    from rt_amd.dist import init_ranks

    init_ranks(dist, backend, torch.device("cuda", device) if backend == "nccl" else None, timeout_s)
    # the ranks that joined the collective: one all-reduce of a 1 per rank
    one = torch.ones(1, dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(one)
    ranks_seen = int(one.item())
    if ranks_seen != world or dist.get_world_size() != world:
        print(f"bench.py: {ranks_seen} ranks joined the all-reduce, WORLD_SIZE={world}", file=sys.stderr,
              flush=True)
        sys.exit(2)
    # distinct GPUs the ranks render on (gloo ranks may share one)
    used = torch.zeros(max(1, torch.cuda.device_count()), dtype=torch.float64, device=one.device)
    used[device] = 1.0
    dist.all_reduce(used, op=dist.ReduceOp.MAX)
    return dist, ranks_seen, int(used.sum().item())


def run_rank(args, ctx_opts, world, rank, local):
    import numpy as np
    import torch

    # one GPU per rank (ranks beyond the visible GPUs share them: gloo only)
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    dist = None
    use_dist = world > 1 or args.force_dist
    ranks_seen, gpus_used = 1, 1
    if use_dist:
        dist, ranks_seen, gpus_used = dist_setup(args.dist_backend, device, world, args.rank_timeout)
    import rt_amd

    name, W, H, depth = CONFIGS[args.config]
    path = scene_path(name)
    scene = rt_amd.Scene(path, W, H, depth)
    t_cold = time.perf_counter()
    ctx = rt_amd.Context(device, **ctx_opts)
    torch.cuda.synchronize()
    t_up = time.perf_counter()
    ctx.upload(scene)  # device copy + cone/cluster prepasses + light-buffer build (synchronous)
    upload_ms = (time.perf_counter() - t_up) * 1e3
    # the process's first frame (cold): upload + first synchronous render of
    # the full frame into pinned host memory
    cold = None
    if world == 1:
        pin = torch.empty((H, W, 4), dtype=torch.uint8).pin_memory()
        t_r = time.perf_counter()
        rt_amd.lib().rt_render(ctx._h, ctypes.byref(scene.frame), pin.data_ptr())
        t_e = time.perf_counter()
        cold = {"first_frame_ms": round((t_e - t_cold) * 1e3, 3), "create_ms": round((t_up - t_cold) * 1e3, 3),
                "upload_ms": round(upload_ms, 3), "first_render_ms": round((t_e - t_r) * 1e3, 3)}
        del pin
    lbinfo = None
    L = rt_amd.lib()
    if hasattr(L, "rt_debug_lb_info"):
        L.rt_debug_lb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        info = (ctypes.c_double * 64)()
        if L.rt_debug_lb_info(ctx._h, info, 64) == 0 and info[0]:
            nl = scene.flat.n_lights
            lbinfo = {"entries": int(info[1]), "build_ms": round(info[2], 2),
                      "cells_per_face_edge": [int(info[3 + 3 * j]) for j in range(min(nl, 20))],
                      "uncullable_pairs": [int(info[4 + 3 * j]) for j in range(min(nl, 20))]}
    types = scene.arrays()[0]
    # compulsory scene bytes: 64-byte surface + 48-byte material records, 32-byte lights
    scene_bytes = int(types.shape[0]) * 112 + int(scene.flat.n_lights) * 32

    from rt_amd.dist import RootGather, band_layout, slab_rows

    r0, r1, rows = slab_rows(H, world, rank)   # equal slabs (padded when H % world != 0)
    frame = scene.frame.copy()
    frame.row_begin, frame.row_end = r0, r1
    stream = torch.cuda.current_stream().cuda_stream
    # Partition: contiguous row slabs, or cyclic 16-row bands
    # when the slabs' render times differ by more than 10% (measured here on
    # every rank before the run; the decision is the same on all ranks).
    partition, imbalance = "slabs", None
    if use_dist and args.partition != "slabs":
        tmp = torch.zeros((max(rows, 1), W, 4), dtype=torch.uint8, device="cuda")
        # the timed loop's kernel: one synchronous render first builds this
        # camera's camera buffer, which the async renders below then use
        ctx.prepare_camera(frame)
        for _ in range(2):
            ctx.render_async(frame, tmp.data_ptr(), 0, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            ctx.render_async(frame, tmp.data_ptr(), 0, stream)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 5
        tmax = torch.tensor([t], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        tsum = tmax.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tsum)
        imbalance = float(tmax.item()) / (float(tsum.item()) / world) - 1.0
        if args.partition == "bands" or imbalance > 0.10:
            partition = "bands"
        del tmp
    band = 16 if partition == "bands" else 0
    if band:
        frame.band_rows, frame.band_count, frame.band_index = band, world, rank
        _, rows = band_layout(H, world, band)
    gather = (RootGather(dist, H, W, "cuda", band_rows=band, batch=args.gather_batch,
                         send_channels=args.gather_channels) if use_dist else None)
    single = torch.zeros((rows, W, 4), dtype=torch.uint8, device="cuda")

    # one counted render (atomics) for the algorithmic work of this rank's slab
    sf = frame.copy()
    sf.flags = rt_amd.FLAG_STATS
    ctx.render(sf)
    st = ctx.stats()
    cbinfo = None  # the camera buffer, built by that synchronous render (per camera)
    if hasattr(L, "rt_debug_cb_info"):
        L.rt_debug_cb_info.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        ci = (ctypes.c_double * 10)()
        if L.rt_debug_cb_info(ctx._h, ci, 10) == 0 and ci[0]:
            cbinfo = {"entries": int(ci[1]), "build_ms": round(ci[2], 3), "tiles": int(ci[3]),
                      "inline_records": bool(ci[4]), "build_host_ms": round(ci[5], 3),
                      "binning": {"candidate_pairs": int(ci[6]), "lists_over_256": int(ci[7]),
                                  "longest_list": int(ci[8]), "capacity": int(ci[9])}}
    brute = algorithmic_flops(types, st.primary_rays, st.bounce_rays, st.shadow_rays)
    flops = executed_flops(st)
    brute_tests = (st.primary_rays + st.bounce_rays + st.shadow_rays) * int(types.shape[0])
    run_tests = st.triangle_tests + st.plane_tests + st.quadric_tests

    counter = [0]
    # the C entry point with its arguments converted once: the Python
    # wrapper's per-call conversions (~10 us) would otherwise bound the
    # launch rate of small frames (C1: 10 us kernels)
    render_async = L.rt_render_async
    c_ctx, c_frame, c_stream = ctx._h, ctypes.byref(frame), ctypes.c_void_p(stream)
    c_single = ctypes.c_void_p(single.data_ptr())

    def step(ev=None):
        k = counter[0]
        counter[0] += 1
        out = ctypes.c_void_p(gather.target(k).data_ptr()) if gather else c_single
        if ev is not None:
            ev[0].record()
        if render_async(c_ctx, c_frame, out, None, c_stream) != 0:
            raise RuntimeError(f"rt_render_async: {ctx._err()}")
        if ev is not None:
            ev[1].record()
        if gather:
            gather.submit(k)   # slab -> rank 0 over xGMI, overlapping the next render

    # Clock settle: untimed renders of this rank's share into a scratch
    # buffer (no gather) until settle_ms of wall time has passed.
    settle_frames, t_settle = 0, time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms and settle_frames < 20000:
        for _ in range(10):
            ctx.render_async(frame, single.data_ptr(), 0, stream)
        settle_frames += 10
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    # Kernel time, measured live over the timed region with HIP events on the
    # stream the kernel is launched on: at N=1 the stream runs nothing but the
    # trace kernel, so one event pair around the K launches / K is the average
    # launch duration (back-to-back, no event packets between launches, which
    # would add their own dispatch latency).  At N>1 the compute stream also
    # waits for gather buffers, so each launch gets its own event pair.
    per_launch = use_dist
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps if per_launch else 1)]
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if not per_launch:
        events[0][0].record()
    for k in range(args.steps):
        step(events[k] if per_launch else None)
    if not per_launch:
        events[0][1].record()
    if gather:
        gather.finish()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the kernel the timed launches ran: rt_stats.kernel of the timed loop's
    # last launch (a camera's first frames compute, then store, its tile
    # masks; the timed frames read them: rt_trace_tiny<0,1,37> at C2)
    timed_kernel = ctx.stats().kernel
    frame_sha = None
    if args.frame_sha and rank == 0:
        import hashlib

        last = gather.frame(args.steps - 1 + args.warmup) if gather else single[:H]
        frame_sha = hashlib.sha256(last.contiguous().cpu().numpy().tobytes()).hexdigest()
    if per_launch:
        kernel_ms = sum(a.elapsed_time(b) for a, b in events) / args.steps
    else:
        kernel_ms = events[0][0].elapsed_time(events[0][1]) / args.steps
    # per-frame kernel times (median beside the mean): after
    # the timed region, K more frames with an event pair around each launch
    frame_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.steps)]
    for a, b in frame_ev:
        a.record()
        ctx.render_async(frame, single.data_ptr(), 0, stream)
        b.record()
    torch.cuda.synchronize()
    per_frame = sorted(a.elapsed_time(b) for a, b in frame_ev)
    ranks_info = None
    if use_dist:
        cdev = "cuda" if args.dist_backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([st.primary_rays, st.bounce_rays, st.shadow_rays], dtype=torch.float64, device=cdev)
        dist.all_reduce(c)
        tot_primary, tot_bounce, tot_shadow = (float(x) for x in c.tolist())
        # The N>1 model's terms: each rank's slab render (median
        # of its per-frame event pairs above) and the gather alone — batches
        # of already-rendered slabs posted back to back after a barrier, with
        # no render beside them, per batch of gather_batch frames.
        nb = 4
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for j in range(nb):
            for i in range(args.gather_batch):
                k = counter[0]
                counter[0] += 1
                gather.target(k)
                gather.submit(k)
        gather.finish()
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3 / nb
        rmed = per_frame[len(per_frame) // 2]
        v = torch.tensor([rmed, -rmed, gather_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        mx, mn, gmax = (float(x) for x in v.tolist())
        ranks_info = {"render_ms_slowest": round(mx, 4), "render_ms_fastest": round(-mn, 4),
                      "gather_ms_per_batch": round(gmax, 4), "gather_batch": args.gather_batch,
                      "bytes_per_link_per_frame": int(rows * W * args.gather_channels),
                      "note": "render: median per-frame launch time of a rank's slab (event pairs), slowest and "
                              "fastest rank; gather: batches of gather_batch already-rendered slabs gathered to "
                              "rank 0 back to back with no render beside them (max over ranks, per batch); bytes: "
                              "one non-root rank's slab per frame over its link to rank 0"}
    else:
        tot_primary, tot_bounce, tot_shadow = float(st.primary_rays), float(st.bounce_rays), float(st.shadow_rays)

    if rank == 0:
        ms = elapsed * 1e3 / args.steps
        value = W * H * args.steps / elapsed / 1e6
        achieved = flops / (kernel_ms * 1e-3) / 1e12
        # Hardware counters of the same kernel on the same config, from the
        # rocprofv3 --pmc passes committed under profiles/ (tools/pmc_summary.py):
        # L2-to-fabric bytes per launch (read requests by size + WRITE_SIZE,
        # calibrated in tools/calib; FETCH_SIZE x2 kept beside it) and VALU
        # wave-instructions per launch; VALU busy = those x 2 cycles (wave64
        # on a SIMD32) over 1,024 SIMDs x this run's kernel time at 2.4 GHz.
        traffic, valu_busy, pmc_src, rec = None, None, None, None
        tfile = os.path.join(REPO, "profiles", "pmc.json")
        if os.path.exists(tfile):
            with open(tfile) as f:
                rec = json.load(f).get(f"{args.config}_n{world}")
            if rec and rec.get("src_sha256") == product_src_sha256():
                traffic = rec.get("hbm_bytes_per_launch")
                if rec.get("SQ_INSTS_VALU"):
                    valu_busy = round(rec["SQ_INSTS_VALU"] * 2 / (1024 * kernel_ms * 1e-3 * 2.4e9), 3)
                pmc_src = rec.get("source")
            elif rec:  # counters of other kernel sources: not this kernel's
                pmc_src = "stale: " + rec.get("source", "") + " (collected on other sources)"
        alg_bytes = 4 * W * rt_amd.frame_rows(frame) + scene_bytes
        out = {
            "metric": "Mray/s and ms/frame at 1920x1080 depth=3, 1/2/4/8 MI355X vs host CPU",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "gpus_used": gpus_used,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"reference scene file {name}" if not name.startswith("heightfield") else
                     "synthetic 50k-triangle heightfield (rt_amd.synth)" +
                     (", reflect 0.5 on every triangle" if name.endswith("_r05") else "")),
            "config": {"workload": f"{name} {W}x{H} max_bounces={depth}", "width": W, "height": H,
                       "max_bounces": depth, "surfaces": int(types.shape[0]),
                       "parallelism": (f"row-band16 x{world}" if band else f"row-slab x{world}") +
                                      ((f" + RCCL gather to rank 0 (double-buffered, {args.gather_batch} frame(s) "
                                        f"per collective, {args.gather_channels} B/px)" if args.dist_backend == "nccl"
                                        else " + gloo gather to rank 0 through host memory") if use_dist else ""),
                       "slab_imbalance": round(imbalance, 3) if imbalance is not None else None,
                       **({"options": ctx_opts} if ctx_opts else {})},
            "total_rays_per_s_M": round((tot_primary + tot_bounce + tot_shadow) * args.steps / elapsed / 1e6, 3),
            "rays_per_frame": {"primary": int(tot_primary), "bounce": int(tot_bounce), "shadow": int(tot_shadow)},
            "bounce_walk": ({"triangle_tests_per_bounce_ray": round(st.bounce_triangle_tests / st.bounce_rays, 2),
                             "bvh_nodes_per_bounce_ray": round(st.bvh_nodes_visited / st.bounce_rays, 2),
                             "triangles": int(np.sum(types == 0)),
                             "note": "this rank's bounce rays (Scene.cpp:1779-1823): exact triangle tests and BVH "
                                     "inner nodes visited per ray (brute force: every triangle)"}
                            if st.bounce_rays else None),
            "kernel_ms": round(kernel_ms, 4),
            "frame_ms": {"median": round(per_frame[len(per_frame) // 2], 4),
                         "mean": round(sum(per_frame) / len(per_frame), 4),
                         "p10": round(per_frame[len(per_frame) // 10], 4),
                         "p90": round(per_frame[(9 * len(per_frame)) // 10], 4), "frames": len(per_frame),
                         "note": "this rank's render of K more frames after the timed region, one HIP event pair "
                                 "around each launch (includes each launch's dispatch gap)"},
            "settle": {"frames": settle_frames, "ms": round(args.settle_ms, 1),
                       "note": "untimed renders before the warmup steps (sustained clock); then warmup, then the "
                               "timed steps"},
            "upload_ms": round(upload_ms, 2),
            "light_buffer": lbinfo,
            "camera_buffer": cbinfo,
            "hbm": {"algorithmic_bytes": int(alg_bytes), "measured_bytes": traffic,
                    "measured_fetch_x2_bytes": (rec or {}).get("fetch_x2_bytes_per_launch") if traffic else None,
                    "measured_note": "L2-to-fabric bytes per launch (Infinity Cache hits included): 128/64/32-B "
                                     "read requests + WRITE_SIZE, calibrated on known-byte kernels (tools/calib)",
                    "measured_gbps": round(traffic / (kernel_ms * 1e-3) / 1e9, 1) if traffic else None,
                    "frac_of_8TBps": round(traffic / (kernel_ms * 1e-3) / 8e12, 4) if traffic else None,
                    "valu_busy": valu_busy, "source": pmc_src},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                         "bound_note": "FP32 VALU-bound (SURVEY 8(d)): priced against the FP32 vector peak, "
                                       "157.3 TF with packed FMA; no dense contraction, so no MFMA instructions",
                         "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
                         "frac_vs_nofma_issue_peak": round(achieved / PEAK_NOFMA_TOPS, 4),
                         "flops_per_launch": int(flops),
                         # the kernel the library reports for the timed loop's last launch
                         # (rt_stats.kernel, ABI 7): the name rocprof's dominant kernel carries
                         "kernel": timed_kernel,
                         "work": "exact ray-primitive tests executed (after culling) x SURVEY 8(d) ops + set-up + shading",
                         "tests_executed": int(run_tests), "tests_brute_force": int(brute_tests),
                         "brute_force_equiv_tflops": round(brute / (kernel_ms * 1e-3) / 1e12, 3)},
        }
        if ranks_info:
            out["ranks"] = ranks_info
        if frame_sha:
            out["frame_rgba8_sha256"] = frame_sha
        if world == 1 and not args.no_host_boundary:
            out["host_boundary"] = host_boundary(ctx, frame, W)
            fc = frame_costs(scene, frame, W, cold, ctx_opts)
            out["first_frame_ms"] = fc.get("first_frame_ms")
            out["moving_camera_ms_per_frame"] = fc.get("moving_camera_ms_per_frame")
            mc = fc.get("moving_camera") or {}
            if mc.get("async_device_ms_per_frame"):
                # the camera moved every frame, device-resident output: the
                # per-frame cost of any use that moves the camera (value
                # re-renders one camera whose per-camera state is built once)
                out["moving_camera_async_ms"] = mc["async_device_ms_per_frame"]
                out["moving_camera_async_mray_s"] = round(W * H / mc["async_device_ms_per_frame"] / 1e3, 3)
                # the same moved cameras, each camera's first frame against its
                # repeats: the per-camera cost without the picture change
                out["moving_camera_same_cameras"] = mc.get("same_cameras")
            out["frame_costs"] = fc
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(path, W, H, depth, args.cpu_seconds)
            cb["gpu_over_cpu"] = round(value / cb["value"], 1) if cb["value"] else None
            out["cpu_baseline"] = cb
            ca = cpu_allcores(path, W, H, depth, max(2.0, args.cpu_seconds / 2))
            ca["gpu_over_cpu"] = round(value / ca["value"], 1) if ca["value"] else None
            out["cpu_baseline_allcores"] = ca
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
