"""cmp_gpu_gather's multi-rank protocol on the CPU (ADVICE r5,
VERDICT r5 weak #5): WORLD ranks as threads of one process, each with its own
engine over the host-memory device stub (tests/sanitize/dev_stub.c) and a
communicator of tests/sanitize/fake_rccl.c (the eight RCCL calls the gather
makes, over host memory), built with ASan + UBSan (tests/sanitize/Makefile,
gather_sim).  For every scenario -- the plain gather, whose root buffer,
table and patched identifiers are checked against the frames, and a refusal
on ONE rank: the root's capacity, alignment or NULL buffer, a peer's NULL
frames, an allocation failing on one rank (the size table, the packing, the
root's identifier table), an error-valued size, a frame that made no draw --
every rank must return the same value, and none may be left waiting inside a
collective (the harness's watchdog fails a run that hangs)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")
GENERIC, PARAMS_INVALID, DST_TOO_SMALL = 2**32 - 1, 2**32 - 10, 2**32 - 30
S_OK, S_ROOT_SMALL, S_ROOT_MISALIGNED, S_ROOT_OUT_NULL, S_PEER_FRAMES_NULL, S_PEER_FAIL_TABLE, \
    S_PEER_FAIL_PACK, S_ROOT_FAIL_TABLE, S_ROOT_FAIL_PATCH, S_ERROR_SIZE, S_NO_DRAW = range(11)


def expected(scenario, layout):
    if scenario == S_OK:
        return 0
    if scenario in (S_ROOT_SMALL, S_ROOT_MISALIGNED):
        return DST_TOO_SMALL
    if scenario == S_NO_DRAW:
        return 0 if layout == 2 else PARAMS_INVALID  # the streams layout keeps such a frame's identifier
    return GENERIC


@pytest.fixture(scope="module")
def sim():
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    r = subprocess.run(["make", "-s", "-C", HERE, "gather_sim"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return os.path.join(HERE, "gather_sim")


@pytest.mark.parametrize("world,root", [(1, 0), (2, 0), (2, 1), (3, 1), (5, 0), (5, 4)])
@pytest.mark.parametrize("layout", [0, 1, 2])
def test_gather_every_rank_same_answer(sim, world, root, layout):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    for scenario in range(11):
        r = subprocess.run([sim, str(world), str(root), str(scenario), str(layout)], capture_output=True, text=True,
                           env=env, timeout=60)
        assert r.returncode == 0, (scenario, r.returncode, r.stderr[-3000:])
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
        rets = [int(v) for v in r.stdout.split()[1:]]
        assert len(rets) == world
        assert rets == [expected(scenario, layout)] * world, (scenario, rets)
