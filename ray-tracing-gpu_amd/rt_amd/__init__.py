"""rt_amd — Python host binding of librt_amd.so (the MI355X ray tracer).

The product is the C ABI in ``include/rt.h``; this module is a thin ctypes
binding over it, shaped like the reference's ``CScene`` (Scene.h:41-70) so a
caller of the reference finds the same verbs:

    scene = CScene()
    scene.AjusterResolution(1920, 1080)        # Scene.cpp:162
    scene.AjusterNbRebondsMax(3)               # Scene.cpp:180
    scene.TraiterFichierDeScene("scene2.dat")  # Scene.cpp:231
    img = scene.LancerRayons()                 # Scene.cpp:672 -> (H, W, 4) uint8, row 0 = bottom

There is no CPU fallback: if ``librt_amd.so`` is missing or no HIP device is
usable, the render calls raise.  Host-only calls (parsing, Pretraitement,
flattening) work without a GPU.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

__all__ = [
    "RtError", "SceneFlat", "Frame", "Stats", "Scene", "Context", "CpuContext", "CScene", "lib", "band_rows",
    "frame_rows",
    "LIB_PATH", "TRIANGLE", "PLANE", "QUADRIC", "FLAG_STATS", "OPTIONS", "camera_path",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "librt_amd.so"))

TRIANGLE, PLANE, QUADRIC = 0, 1, 2
FLAG_STATS = 1
# rt.h RT_OPT_* (ABI 5): A/B and test switches, none changes an image bit
OPTIONS = {"light_buffer": 1, "camera_buffer": 2, "union_pretest": 3, "lb_scale": 4, "dcov_near": 5,
           "cb_inline_max_mb": 6, "host_chunk_mb": 7, "cb_capacity": 8, "launch_camera": 12, "bvh": 13, "wavefront": 14,
           "wf_sort": 15, "xcd_deal": 16, "xcd_stripe": 17, "lb_unroll": 18, "wf_overlap": 19}
_ERRORS = {-1: "RT_E_ARG", -2: "RT_E_IO", -3: "RT_E_PARSE", -4: "RT_E_STATE", -5: "RT_E_HIP",
           -6: "RT_E_UNSUPPORTED"}


class RtError(RuntimeError):
    def __init__(self, where: str, code: int, msg: str = ""):
        super().__init__(f"{where} failed: {_ERRORS.get(code, code)} {msg}".rstrip())
        self.code = code


class SceneFlat(ctypes.Structure):
    _fields_ = [("n_surfaces", ctypes.c_int32), ("n_lights", ctypes.c_int32),
                ("type", ctypes.POINTER(ctypes.c_int32)), ("geom", ctypes.POINTER(ctypes.c_float)),
                ("material", ctypes.POINTER(ctypes.c_float)), ("lights", ctypes.POINTER(ctypes.c_float))]


class Frame(ctypes.Structure):
    _fields_ = [("cam_pos", ctypes.c_float * 3), ("orient", ctypes.c_float * 16),
                ("half_w", ctypes.c_float), ("half_h", ctypes.c_float),
                ("inv_w", ctypes.c_float), ("inv_h", ctypes.c_float),
                ("background", ctypes.c_float * 3),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("row_begin", ctypes.c_int32), ("row_end", ctypes.c_int32),
                ("max_bounces", ctypes.c_int32), ("min_energy", ctypes.c_float),
                ("scene_ior", ctypes.c_float), ("flags", ctypes.c_int32),
                ("band_rows", ctypes.c_int32), ("band_count", ctypes.c_int32), ("band_index", ctypes.c_int32)]

    def copy(self) -> "Frame":
        f = Frame()
        ctypes.pointer(f)[0] = self
        return f


class Stats(ctypes.Structure):
    _fields_ = [("primary_rays", ctypes.c_uint64), ("bounce_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("shadow_tests_skipped", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_float), ("stack_depth", ctypes.c_int32),
                ("light_batch", ctypes.c_int32), ("triangle_tests", ctypes.c_uint64),
                ("plane_tests", ctypes.c_uint64), ("quadric_tests", ctypes.c_uint64),
                ("bounce_triangle_tests", ctypes.c_uint64), ("bvh_nodes_visited", ctypes.c_uint64),
                ("kernel_name", ctypes.c_char * 48)]

    @property
    def kernel(self) -> str:
        """The trace kernel that ran (rt_stats.kernel)."""
        return self.kernel_name.decode()


_lib: Optional[ctypes.CDLL] = None

# Every symbol include/rt.h declares, with its ctypes signature.
_VP = ctypes.c_void_p
SIGNATURES = {
    "rt_abi_version": (ctypes.c_int, []),
    "rt_band_rows": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "rt_scene_create": (ctypes.c_int, [ctypes.POINTER(_VP)]),
    "rt_scene_set_resolution": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_int32]),
    "rt_scene_set_max_bounces": (ctypes.c_int, [_VP, ctypes.c_int32]),
    "rt_scene_set_min_energy": (ctypes.c_int, [_VP, ctypes.c_float]),
    "rt_scene_set_scene_ior": (ctypes.c_int, [_VP, ctypes.c_float]),
    "rt_scene_load_file": (ctypes.c_int, [_VP, ctypes.c_char_p]),
    "rt_scene_prepare": (ctypes.c_int, [_VP]),
    "rt_scene_get_flat": (ctypes.c_int, [_VP, ctypes.POINTER(SceneFlat)]),
    "rt_scene_get_frame": (ctypes.c_int, [_VP, ctypes.POINTER(Frame)]),
    "rt_scene_error": (ctypes.c_char_p, [_VP]),
    "rt_scene_destroy": (None, [_VP]),
    "rt_create": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_VP)]),
    "rt_create_cpu": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_VP)]),
    "rt_cpu_render": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), _VP]),
    "rt_cpu_render_float": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), _VP]),
    "rt_upload_scene": (ctypes.c_int, [_VP, ctypes.POINTER(SceneFlat)]),
    "rt_render": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), _VP]),
    "rt_render_float": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), _VP]),
    "rt_render_async": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), _VP, _VP, _VP]),
    "rt_prepare_camera": (ctypes.c_int, [_VP, ctypes.POINTER(Frame)]),
    "rt_render_sequence_async": (ctypes.c_int, [_VP, ctypes.POINTER(Frame), ctypes.c_int32, _VP, ctypes.c_size_t, _VP,
                                                ctypes.c_size_t, _VP]),
    "rt_sync": (ctypes.c_int, [_VP]),
    "rt_set_option": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.c_double]),
    "rt_get_option": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]),
    "rt_set_far_ladder": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double), ctypes.c_int32]),
    "rt_last_stats": (ctypes.c_int, [_VP, ctypes.POINTER(Stats)]),
    "rt_last_error": (ctypes.c_char_p, [_VP]),
    "rt_destroy": (None, [_VP]),
}


def band_rows(height: int, band_rows: int, band_count: int, band_index: int) -> int:
    """Output rows of one rank's cyclic band set (rt.h rt_band_rows), host-side."""
    if height < 0 or band_rows <= 0 or band_rows % 16 or band_count <= 0 or not 0 <= band_index < band_count:
        raise ValueError("bad band layout")
    nb = -(-height // band_rows)
    return (-(-(nb - band_index) // band_count) if nb > band_index else 0) * band_rows


def frame_rows(frame: "Frame") -> int:
    """Rows a render of `frame` writes: the slab, or the packed band set."""
    if frame.band_rows:  # an invalid layout gives 0 rows here; the render call rejects it
        return max(0, lib().rt_band_rows(frame.height, frame.band_rows, frame.band_count, frame.band_index))
    return frame.row_end - frame.row_begin


def lib() -> ctypes.CDLL:
    """Load librt_amd.so once; raise (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: when PyTorch (the device-memory /
        # stream / RCCL plumbing) is installed, its bundled libamdhip64.so.7
        # must be the one librt_amd.so binds to (same SONAME), so load it first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RtError("load", -4, f"{LIB_PATH} not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(where: str, rc: int, msg_fn=None):
    if rc != 0:
        raise RtError(where, rc, msg_fn() if msg_fn else "")


class Scene:
    """Host scene: CScene's parser + Initialiser (camera, Pretraitement)."""

    def __init__(self, path: str, width: int, height: int, max_bounces: int = 0,
                 min_energy: float = 0.01, scene_ior: float = 1.0):
        L = lib()
        self._h = _VP()
        _check("rt_scene_create", L.rt_scene_create(ctypes.byref(self._h)))
        err = lambda: (L.rt_scene_error(self._h) or b"").decode()
        _check("rt_scene_set_resolution", L.rt_scene_set_resolution(self._h, width, height), err)
        _check("rt_scene_set_max_bounces", L.rt_scene_set_max_bounces(self._h, max_bounces), err)
        L.rt_scene_set_min_energy(self._h, min_energy)
        L.rt_scene_set_scene_ior(self._h, scene_ior)
        _check("rt_scene_load_file", L.rt_scene_load_file(self._h, os.fsencode(path)), err)
        _check("rt_scene_prepare", L.rt_scene_prepare(self._h), err)
        self.flat = SceneFlat()
        _check("rt_scene_get_flat", L.rt_scene_get_flat(self._h, ctypes.byref(self.flat)))
        self.frame = Frame()
        _check("rt_scene_get_frame", L.rt_scene_get_frame(self._h, ctypes.byref(self.frame)))
        self.width, self.height = width, height

    @property
    def n_surfaces(self) -> int:
        return self.flat.n_surfaces

    def arrays(self):
        """(type[n], geom[n,12], material[n,10], lights[L,7]) as numpy copies."""
        n, nl = self.flat.n_surfaces, self.flat.n_lights
        t = np.ctypeslib.as_array(self.flat.type, (max(n, 1),))[:n].copy() if n else np.zeros(0, np.int32)
        g = np.ctypeslib.as_array(self.flat.geom, (max(n, 1) * 12,))[: n * 12].reshape(n, 12).copy() if n else np.zeros((0, 12), np.float32)
        m = np.ctypeslib.as_array(self.flat.material, (max(n, 1) * 10,))[: n * 10].reshape(n, 10).copy() if n else np.zeros((0, 10), np.float32)
        l = np.ctypeslib.as_array(self.flat.lights, (max(nl, 1) * 7,))[: nl * 7].reshape(nl, 7).copy() if nl else np.zeros((0, 7), np.float32)
        return t, g, m, l

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One HIP device: uploaded scene + render entry points."""

    def __init__(self, device: int = 0, **options):
        L = lib()
        self._h = _VP()
        rc = L.rt_create(device, ctypes.byref(self._h))
        if rc != 0:
            msg = (L.rt_last_error(self._h) or b"").decode() if self._h else ""
            if self._h:
                L.rt_destroy(self._h)
                self._h = None
            raise RtError("rt_create", rc, msg)
        for k, v in options.items():
            if k == "far_ladder":
                self.set_far_ladder(v)
            else:
                self.set_option(k, v)

    def set_option(self, name, value: float):
        """rt_set_option: `name` is a key of OPTIONS (or the RT_OPT_* number)."""
        opt = OPTIONS[name] if isinstance(name, str) else int(name)
        _check("rt_set_option", lib().rt_set_option(self._h, opt, float(value)), self._err)

    def get_option(self, name) -> float:
        opt = OPTIONS[name] if isinstance(name, str) else int(name)
        v = ctypes.c_double()
        _check("rt_get_option", lib().rt_get_option(self._h, opt, ctypes.byref(v)), self._err)
        return v.value

    def set_far_ladder(self, factors=None):
        """rt_set_far_ladder: the big lists' far light buffers (None = default)."""
        if factors is None:
            _check("rt_set_far_ladder", lib().rt_set_far_ladder(self._h, None, -1), self._err)
            return
        arr = (ctypes.c_double * max(1, len(factors)))(*factors)
        _check("rt_set_far_ladder", lib().rt_set_far_ladder(self._h, arr, len(factors)), self._err)

    def render_sequence_async(self, frames, rgba_dev_ptr: int = 0, rgba_stride: int = 0, rgb_dev_ptr: int = 0,
                              rgb_stride: int = 0, stream: int = 0):
        """rt_render_sequence_async: a camera path enqueued on `stream`."""
        arr = (Frame * max(1, len(frames)))(*frames)
        _check("rt_render_sequence_async",
               lib().rt_render_sequence_async(self._h, arr, len(frames), rgba_dev_ptr or None, rgba_stride,
                                              rgb_dev_ptr or None, rgb_stride, stream or None), self._err)

    def prepare_camera(self, frame: Frame):
        _check("rt_prepare_camera", lib().rt_prepare_camera(self._h, ctypes.byref(frame)), self._err)

    def sync(self):
        _check("rt_sync", lib().rt_sync(self._h), self._err)

    def _err(self) -> str:
        return (lib().rt_last_error(self._h) or b"").decode()

    def upload(self, scene: Scene):
        _check("rt_upload_scene", lib().rt_upload_scene(self._h, ctypes.byref(scene.flat)), self._err)

    def render(self, frame: Frame) -> np.ndarray:
        """RGBA8 (rows, W, 4), row 0 = frame.row_begin (bottom-up), or this
        rank's packed band set when frame.band_rows > 0."""
        rows = frame_rows(frame)
        out = np.zeros((rows, frame.width, 4), np.uint8)
        _check("rt_render", lib().rt_render(self._h, ctypes.byref(frame), out.ctypes.data), self._err)
        return out

    def render_float(self, frame: Frame) -> np.ndarray:
        rows = frame_rows(frame)
        out = np.zeros((rows, frame.width, 3), np.float32)
        _check("rt_render_float", lib().rt_render_float(self._h, ctypes.byref(frame), out.ctypes.data), self._err)
        return out

    def render_async(self, frame: Frame, rgba_dev_ptr: int = 0, rgb_dev_ptr: int = 0, stream: int = 0):
        _check("rt_render_async", lib().rt_render_async(self._h, ctypes.byref(frame), rgba_dev_ptr or None,
                                                        rgb_dev_ptr or None, stream or None), self._err)

    def stats(self) -> Stats:
        s = Stats()
        _check("rt_last_stats", lib().rt_last_stats(self._h, ctypes.byref(s)))
        return s

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def camera_path(frame: Frame, n: int, yaw_deg: float = 0.5, step=(0.4, 0.0, -0.25)):
    """n frames of a camera path from `frame`: each step yaws the camera by
    yaw_deg about its own up axis (orientation rows U, V, N — Scene.cpp:
    624-660) and moves it by `step` (world units); returns new Frames."""
    out = []
    o = np.array(frame.orient[:], np.float64).reshape(4, 4)
    pos = np.array(frame.cam_pos[:], np.float64)
    for k in range(n):
        a = np.deg2rad(yaw_deg * k)
        U, N = o[0, :3], o[2, :3]
        m = o.copy()
        m[0, :3] = np.cos(a) * U - np.sin(a) * N
        m[2, :3] = np.sin(a) * U + np.cos(a) * N
        f = frame.copy()
        for i, v in enumerate(m.astype(np.float32).ravel()):
            f.orient[i] = float(v)
        p = (pos + k * np.array(step)).astype(np.float32)
        f.cam_pos[0], f.cam_pos[1], f.cam_pos[2] = (float(x) for x in p)
        out.append(f)
    return out


class CpuContext:
    """The CPU backend (rt_create_cpu / rt_cpu_render*): the same images on
    host threads.  Explicit only — Context never falls back to it."""

    def __init__(self, threads: int = 0):
        L = lib()
        self._h = _VP()
        _check("rt_create_cpu", L.rt_create_cpu(threads, ctypes.byref(self._h)))

    def _err(self) -> str:
        return (lib().rt_last_error(self._h) or b"").decode()

    def upload(self, scene: Scene):
        _check("rt_upload_scene", lib().rt_upload_scene(self._h, ctypes.byref(scene.flat)), self._err)

    def render(self, frame: Frame) -> np.ndarray:
        out = np.zeros((frame_rows(frame), frame.width, 4), np.uint8)
        _check("rt_cpu_render", lib().rt_cpu_render(self._h, ctypes.byref(frame), out.ctypes.data), self._err)
        return out

    def render_float(self, frame: Frame) -> np.ndarray:
        out = np.zeros((frame_rows(frame), frame.width, 3), np.float32)
        _check("rt_cpu_render_float", lib().rt_cpu_render_float(self._h, ctypes.byref(frame), out.ctypes.data),
               self._err)
        return out

    def stats(self) -> Stats:
        s = Stats()
        _check("rt_last_stats", lib().rt_last_stats(self._h, ctypes.byref(s)))
        return s

    def close(self):
        if getattr(self, "_h", None):
            lib().rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CScene:
    """The reference's CScene verbs (Scene.h:41-70) over the HIP backend, or —
    backend="cpu", the reference's CVar::g_ComputerShadersON = false — the
    CPU backend."""

    def __init__(self, device: int = 0, backend: str = "hip", threads: int = 0):
        if backend not in ("hip", "cpu"):
            raise ValueError("backend is 'hip' or 'cpu'")
        self._backend, self._threads = backend, threads
        self._w, self._h = 512, 256          # Var.cpp:4-5
        self._max_bounces = 20               # Scene.cpp:68
        self._min_energy = 0.01              # Scene.cpp:69
        self._scene_ior = 1.0                # Scene.cpp:70
        self._path: Optional[str] = None
        self._device = device
        self._scene: Optional[Scene] = None
        self._ctx: Optional[Context] = None

    def AjusterResolution(self, w: int, h: int):
        self._w, self._h = int(w), int(h)
        self._scene = None

    def AjusterNbRebondsMax(self, n: int):
        self._max_bounces = int(n)

    def AjusterEnergieMinimale(self, e: float):
        self._min_energy = float(e)

    def AjusterIndiceRefraction(self, ior: float):
        self._scene_ior = float(ior)

    def TraiterFichierDeScene(self, path: str):
        self._path = path
        self._scene = None

    def _prepared(self) -> Scene:
        if self._path is None:
            raise RtError("LancerRayons", -4, "no scene file (TraiterFichierDeScene)")
        if self._scene is None:
            self._scene = Scene(self._path, self._w, self._h, self._max_bounces, self._min_energy, self._scene_ior)
            if self._ctx is None:
                self._ctx = Context(self._device) if self._backend == "hip" else CpuContext(self._threads)
            self._ctx.upload(self._scene)
        return self._scene

    def _frame(self) -> Frame:
        f = self._prepared().frame.copy()
        f.max_bounces, f.min_energy, f.scene_ior = self._max_bounces, self._min_energy, self._scene_ior
        return f

    def LancerRayons(self) -> np.ndarray:
        """Render the frame; returns RGBA8 (H, W, 4), row 0 = bottom."""
        f = self._frame()
        return self._ctx.render(f)

    def LancerRayonsFloat(self) -> np.ndarray:
        """m_InfoPixel equivalent: float32 (H, W, 3), unclamped."""
        f = self._frame()
        return self._ctx.render_float(f)
