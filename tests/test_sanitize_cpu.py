"""SURVEY.md section 5, sanitizer row: the host C code of libairscmp.so
(cmp_host.c: argument checks, the context state machine, the batch planner
with its step-by-step fallback path) and the CLI --params parser built with
AddressSanitizer + UndefinedBehaviorSanitizer (tests/sanitize/Makefile) and
driven by tests/sanitize/host_fuzz.c over pseudo-random valid and invalid
inputs.  The device layer is a host-memory stub (tests/sanitize/dev_stub.c),
so this runs on the CPU; the GPU kernels are covered by the -m gpu tests."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.fixture(scope="module")
def fuzz_bin():
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-s", "-C", HERE, "host_fuzz"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return os.path.join(HERE, "host_fuzz")


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_host_code_clean_under_asan_ubsan(fuzz_bin, seed):
    # (verify_asan_link_order=0: the environment may preload a library ahead
    # of the ASan runtime; it is left as it is)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz_bin, "5000", str(seed)], capture_output=True, text=True, errors="replace", env=env, timeout=600)
    report = "\n".join(l for l in r.stderr.splitlines() if not l.startswith("airspace:"))
    assert r.returncode == 0, report[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, report[-4000:]
    m = re.search(r"(\d+) contexts initialised, host frames (\d+) ok / (\d+) errors, (\d+) batches "
                  r"\((\d+) frames ok, (\d+) with fallback.* (\d+) walks", r.stdout)
    assert m, r.stdout
    init, ok, err, batches, bframes, fb, walks = map(int, m.groups())
    # the run reached the compress paths, their error paths, the planner and
    # the MODEL walk (airs_dev_walk)
    assert init > 1000 and ok > 1000 and err > 100 and batches > 1000 and fb > 300 and walks > 5, m.group(0)
