"""The C ABI boundary: librt_amd.so loads and exports every symbol that
include/rt.h declares, struct layouts agree with the header, and argument
errors come back as codes (never exits).  No compute calls: CPU only."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest

import rt_amd
from conftest import REPO

HEADER = os.path.join(REPO, "include", "rt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 20
    L = rt_amd.lib()
    for n in names:
        assert hasattr(L, n), n
    # the ctypes binding covers exactly the header
    assert set(names) == set(rt_amd.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", rt_amd.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n


def test_every_export_is_declared():
    """No undocumented exports: every rt_* symbol of the library is declared in
    include/rt.h (the boundary) or include/rt_debug.h (diagnostics), and
    rt_debug.h's symbols outside its RT_PROF block are exported."""
    dbg = open(os.path.join(REPO, "include", "rt_debug.h")).read()
    dbg = re.sub(r"/\*.*?\*/", "", dbg, flags=re.S)
    dbg_all = set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", dbg))
    dbg_plain = set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", re.sub(r"#ifdef RT_PROF.*?#endif", "", dbg, flags=re.S)))
    out = subprocess.run(["nm", "-D", "--defined-only", rt_amd.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rt_[a-z_0-9]+)\b", out))
    assert exported <= set(declared_functions()) | dbg_all, exported - set(declared_functions()) - dbg_all
    assert dbg_plain <= exported, dbg_plain - exported


def test_gather_library_exports_its_header():
    """librt_gather.so (the frame's RCCL gather, include/rt_gather.h) exports
    exactly the functions its header declares, and links RCCL."""
    hdr = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "rt_gather.h")).read(), flags=re.S)
    declared = set(re.findall(r"\b(rt_gather_[a-z_0-9]*)\s*\(", hdr))
    lib = os.path.join(REPO, "ray-tracing-gpu_amd", "lib", "librt_gather.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rt_[a-z_0-9]+)\b", out))
    assert exported == declared, (exported ^ declared)
    deps = subprocess.run(["objdump", "-p", lib], capture_output=True, text=True).stdout
    assert "librccl.so" in deps
    # the renderer itself never links RCCL (PyTorch brings its own)
    assert "librccl" not in subprocess.run(["objdump", "-p", rt_amd.LIB_PATH], capture_output=True, text=True).stdout
    # rt_render loads librt_gather.so (and RCCL) only on its RCCL path (dlopen)
    exe = os.path.join(REPO, "ray-tracing-gpu_amd", "lib", "rt_render")
    needed = subprocess.run(["objdump", "-p", exe], capture_output=True, text=True).stdout
    assert "librt_gather" not in needed and "librccl" not in needed


def test_abi_version():
    assert rt_amd.lib().rt_abi_version() == 8


def test_struct_layouts_match_header():
    src = r"""
#include <stdio.h>
#include <stddef.h>
#include "rt.h"
int main(void){
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(rt_scene_flat), sizeof(rt_frame), sizeof(rt_stats),
         offsetof(rt_frame, width), offsetof(rt_frame, flags), offsetof(rt_stats, kernel_ms),
         offsetof(rt_stats, triangle_tests), offsetof(rt_frame, band_index));
  return 0; }
"""
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        vals = list(map(int, subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()))
    assert vals == [ctypes.sizeof(rt_amd.SceneFlat), ctypes.sizeof(rt_amd.Frame), ctypes.sizeof(rt_amd.Stats),
                    rt_amd.Frame.width.offset, rt_amd.Frame.flags.offset, rt_amd.Stats.kernel_ms.offset,
                    rt_amd.Stats.triangle_tests.offset, rt_amd.Frame.band_index.offset]


def test_null_arguments_are_errors():
    L = rt_amd.lib()
    assert L.rt_scene_create(None) == -1
    assert L.rt_scene_set_resolution(None, 4, 4) == -1
    assert L.rt_scene_load_file(None, b"x") == -1
    assert L.rt_upload_scene(None, None) == -1
    assert L.rt_render(None, None, None) == -1
    assert L.rt_render_float(None, None, None) == -1
    assert L.rt_render_async(None, None, None, None, None) == -1
    assert L.rt_last_stats(None, None) == -1
    assert L.rt_prepare_camera(None, None) == -1
    assert L.rt_sync(None) == -1
    assert L.rt_set_option(None, 1, 0.0) == -1
    assert L.rt_get_option(None, 1, None) == -1
    assert L.rt_set_far_ladder(None, None, 0) == -1
    assert L.rt_last_error(None) == b"null context"
    L.rt_destroy(None)
    L.rt_scene_destroy(None)


def test_call_order_errors():
    L = rt_amd.lib()
    h = ctypes.c_void_p()
    assert L.rt_scene_create(ctypes.byref(h)) == 0
    f = rt_amd.SceneFlat()
    assert L.rt_scene_get_flat(h, ctypes.byref(f)) == -4      # before prepare
    assert L.rt_scene_prepare(h) == -4                         # before load
    assert L.rt_scene_set_max_bounces(h, -1) == -1
    L.rt_scene_destroy(h)


def test_cli_built():
    exe = os.path.join(REPO, "ray-tracing-gpu_amd", "lib", "rt_render")
    assert os.access(exe, os.X_OK)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "Aucune fichier" in r.stderr


def test_band_rows_matches_binding():
    L = rt_amd.lib()
    for h in (1, 15, 16, 17, 1080, 4320):
        for br in (16, 32, 48):
            for n in (1, 2, 3, 8):
                tot = 0
                for i in range(n):
                    got = L.rt_band_rows(h, br, n, i)
                    assert got == rt_amd.band_rows(h, br, n, i)
                    tot += got
                assert tot == -(-h // br) * br  # every band exactly once
    assert L.rt_band_rows(100, 8, 2, 0) == -1    # not a multiple of 16
    assert L.rt_band_rows(100, 16, 2, 2) == -1   # index out of range


def test_option_enum_matches_binding_and_round_trips():
    """Every RT_OPT_* of include/rt.h is in rt_amd.OPTIONS under its lower-case
    name with the same number, and rt_set_option / rt_get_option round-trip
    each on a CPU context (the setter is host code: no GPU needed)."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    enum = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"\bRT_OPT_([A-Z0-9_]+)\s*=\s*(\d+)", text)}
    assert enum == rt_amd.OPTIONS
    L = rt_amd.lib()
    h = ctypes.c_void_p()
    assert L.rt_create_cpu(1, ctypes.byref(h)) == 0
    values = {"light_buffer": 2, "camera_buffer": 2, "union_pretest": 0, "lb_scale": 8, "dcov_near": 1.5,
              "cb_inline_max_mb": 64, "host_chunk_mb": 4, "cb_capacity": 1000, "launch_camera": 0, "bvh": 0, "wavefront": 0,
              "wf_sort": 0, "xcd_deal": 3, "xcd_stripe": 4,
              "lb_unroll": 0, "wf_overlap": 0}
    assert set(values) == set(enum)
    try:
        for name, v in values.items():
            assert L.rt_set_option(h, enum[name], ctypes.c_double(v)) == 0, name
            got = ctypes.c_double()
            assert L.rt_get_option(h, enum[name], ctypes.byref(got)) == 0, name
            assert got.value == v, name
        assert L.rt_set_option(h, 999, ctypes.c_double(1)) != 0
        for removed in (9, 10, 11):  # ABI 5's set-aside options (rt.h)
            assert L.rt_set_option(h, removed, ctypes.c_double(1)) != 0
    finally:
        L.rt_destroy(h)
