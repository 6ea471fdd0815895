"""The device prefix sum every on-stream build uses (rt_scan.h: the
camera-buffer tile and triangle offsets, the light-buffer cell offsets):
exclusive prefixes mod 2^32 and a 64-bit total, in place, for the one-block
path (n <= 65,536) and the three-pass path, against numpy."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import rt_amd

pytestmark = pytest.mark.gpu


def _scan(counts):
    L = rt_amd.lib()
    L.rt_debug_scan.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    a = np.ascontiguousarray(counts, dtype=np.uint32)
    out = np.zeros(a.size + 1, np.uint32)
    tot = ctypes.c_ulonglong()
    assert L.rt_debug_scan(0, a.ctypes.data, a.size, out.ctypes.data, ctypes.byref(tot)) == 0
    return out, tot.value


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 1000, 1023, 1024, 1025, 32400, 50176, 65535, 65536, 65537,
                               200000])
@pytest.mark.parametrize("big", [False, True])
def test_scan_matches_numpy(n, big):
    rng = np.random.default_rng(n + 7 * big)
    hi = 2**32 - 1 if big else 300
    a = rng.integers(0, hi, size=n, dtype=np.uint64).astype(np.uint32)
    if n > 3:
        a[rng.integers(0, n, size=n // 4)] = 0  # empty runs, like most tiles' counts
    out, tot = _scan(a)
    ex = np.concatenate([[0], np.cumsum(a.astype(np.uint64))])
    assert tot == int(ex[-1])
    assert np.array_equal(out, (ex % 2**32).astype(np.uint32))
