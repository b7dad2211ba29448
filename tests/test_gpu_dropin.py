"""Literal drop-in evidence for the cmp.h boundary: the reference's own
example caller, examples/simple_compression.c (:58-322), compiled UNCHANGED
from the reference tree against include/ and linked to libairscmp.so
(tests/dropin/Makefile, built by __graft_entry__.build() where the reference
is present), runs on the GPU and prints the two frames the reference prints
(tests/golden/kats.json "simple_compression_example", written by the
reference compiled from its own sources)."""
import json
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "dropin", "simple_compression")


def test_reference_example_links_and_matches(prod):
    if not os.path.exists(BIN):
        pytest.skip("tests/dropin/simple_compression not built (the reference tree was absent at build time)")
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # "1st Compressed Data (Size: 26 bytes):" then hex bytes, 32 per line
    blocks = re.findall(r"Compressed Data \(Size: (\d+) bytes\):\n((?:[0-9A-F]{2}[ \n])+)", r.stdout)
    assert len(blocks) == 2, r.stdout
    with open(os.path.join(ROOT, "tests", "golden", "kats.json")) as f:
        case = next(c for c in json.load(f)["cases"] if c["name"] == "simple_compression_example")
    for (size, hexes), want in zip(blocks, case["expect_frames"]):
        got = "".join(hexes.split())
        assert int(size) * 2 == len(got)
        assert got == want, (got, want)
    # the binary really ran on this library (not a reference build)
    ldd = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libairscmp.so" in ldd, ldd
