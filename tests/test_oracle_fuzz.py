"""The oracle restatement against the reference's own compiled code
(oracle/_ref, built by `make -C oracle ref` in the build container) on the
seeded random scenes of tests/fuzz_scenes.py, bit for bit (skipped where
_ref is not built: the GPU box).  Pins the oracle that tests/test_gpu_fuzz.py
compares the product with."""
from __future__ import annotations

import os
import sys

import pytest

from conftest import REPO, bits_equal
from fuzz_scenes import fuzz_dat

REF = os.path.join(REPO, "oracle", "_ref", "libref_oracle.so")


@pytest.fixture(scope="module")
def ref_lib():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref not built")
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import make_golden

    return make_golden


@pytest.mark.parametrize("seed", range(120))
def test_oracle_matches_reference_on_fuzz_scenes(oracle, ref_lib, tmp_path, seed):
    big = seed % 10 == 7
    path = tmp_path / f"fuzz{seed}.dat"
    path.write_text(fuzz_dat(seed, seed % 3 == 2, big))
    depth = 0 if big and seed % 20 == 7 else seed % 6
    w, h = (64, 48) if big else (48, 36)
    want = ref_lib.Ref(ref_lib.load_ref(), str(path), w, h, depth).window(0, h, 0, w)
    assert bits_equal(oracle.render(str(path), w, h, depth), want)
