"""Host AddressSanitizer + UBSan over the parsers of untrusted scene text
(SURVEY.md §5): the product's loader + Pretraitement (rt_scene.cpp, via the
rt_scene_* C ABI) and the oracle restatement (rt_oracle.c, loader + a small
render), built by tools/sanitize/Makefile with -fno-sanitize-recover=all and
driven over every scene, every loader-quirk file and a heightfield, each
with deterministic mutations (byte flips, truncation, long lines, NaN and
huge numbers, bad point indices).  Any sanitizer report fails the run."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import REPO, SCENES
from loader_quirks import QUIRKS

SAN = os.path.join(REPO, "tools", "sanitize")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-s", "-C", SAN], check=True, timeout=300)
    return os.path.join(SAN, "sanitize_loader")


def test_loaders_under_asan_ubsan(driver, tmp_path):
    from rt_amd import synth

    files = [os.path.join(SCENES, f"scene{i}.dat") for i in range(1, 10)]
    for name, text in QUIRKS.items():
        p = tmp_path / f"{name}.dat"
        p.write_bytes(text.encode())
        files.append(str(p))
    files.append(synth.write_heightfield(str(tmp_path / "hf.dat"), cols=30, rows=12))
    env = dict(os.environ, TMPDIR=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([driver, "300"] + files, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "no sanitizer report" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
