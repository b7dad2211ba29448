"""The arena kernel (airs-compression_amd/csrc/enc_arena.hip): the Rice/ZERO
fast path for 16-bit frames of whole 16 Ki-sample segments (NONE or DIFF,
GOLOMB_ZERO g = 2^k, k <= 11, no model).  Every case is a cmp_gpu_compress
batch compared with the oracle's call loop (include/cmp_gpu.h): frames, sizes
and context state, bit-exact.  Cases cover every k the kernel takes, both
sample types, checksums, several contexts, and segments that do not fit the
arena (incompressible data: the one-chunk-per-pass path) next to segments
that do, inside one frame.

The arena kernel is an experiment, off by default (measured slower than
encode_kernel): every case here turns it on with AIRS_ARENA=1,
which the library reads at each launch."""
import random

import numpy as np
import pytest

import batch_scenarios as bs
from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi
SEG = 16384  # samples per segment of the arena kernel (enc_arena.hip ASEGN)


@pytest.fixture(autouse=True)
def arena_on(monkeypatch):
    monkeypatch.setenv("AIRS_ARENA", "1")


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


def _signal(rng, n, kind, style):
    """16-bit test signals: smooth walks, walks with outliers, noise (about
    16 bits per sample after any predictor: too large for the arena), and a
    frame whose segments alternate between smooth and noise."""
    if style == "smooth":
        x = np.cumsum(rng.integers(-40, 40, n))
    elif style == "outliers":
        x = np.cumsum(rng.integers(-300, 300, n))
        x[rng.integers(0, n, n // 40)] = rng.integers(0, 65536, n // 40)
    elif style == "noise":
        x = rng.integers(0, 65536, n)
    elif style == "zeros":
        x = np.zeros(n, dtype=np.int64)
    else:  # "mixed": segment s is noise for odd s
        x = np.cumsum(rng.integers(-20, 20, n))
        for s in range(1, n // SEG, 2):
            x[s * SEG:(s + 1) * SEG] = rng.integers(0, 65536, SEG)
    x = (x & 0xFFFF).astype(np.uint16)
    return x.view(np.int16) if kind == "i16" else x


CASES = []
for _k in range(12):
    CASES.append((_k, "u16", 1, "smooth"))
CASES += [(5, "i16", 1, "outliers"), (5, "u16", 0, "outliers"), (3, "i16", 0, "smooth"), (0, "u16", 1, "noise"),
          (5, "u16", 1, "noise"), (11, "i16", 1, "noise"), (5, "u16", 1, "mixed"), (2, "i16", 0, "mixed"),
          (0, "u16", 0, "zeros"), (7, "u16", 1, "zeros")]


@pytest.mark.parametrize("k,kind,pre,style", CASES, ids=[f"k{c[0]}-{c[1]}-pre{c[2]}-{c[3]}" for c in CASES])
def test_arena_batch_vs_call_loop(prod, eng, orc, k, kind, pre, style):
    rng = np.random.default_rng(1000 * k + 10 * pre + len(style) + (kind == "i16"))
    r = random.Random(k * 31 + pre)
    n = SEG * r.choice([1, 2, 5])
    nctx, fpc = r.choice([1, 2]), r.choice([1, 3])
    params = api.CmpParams(primary_preprocessing=pre, primary_encoder_type=1, primary_encoder_param=1 << k,
                           checksum_enabled=int(k % 3 == 1))
    srcs = [_signal(rng, n, kind, style) for _ in range(nctx * fpc)]
    cap = 26 + 6 * n  # the worst case: the asynchronous path, one launch
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs)
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs)
    assert got == want


def test_arena_capacity_too_small_vs_call_loop(prod, eng, orc):
    """Capacities below the frame size: the buffer range of the stores drops
    exactly the words past the capacity, and the frames fail with
    DST_TOO_SMALL as in the call loop (the batch steps frame by frame)."""
    rng = np.random.default_rng(7)
    n = 2 * SEG
    params = api.CmpParams(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32)
    srcs = [_signal(rng, n, "u16", s) for s in ("smooth", "noise", "mixed")]
    for cap in (40, 22 + n // 4 + 3, 22 + n + 1, 26 + 3 * n):
        want = bs.run_batch_host(orc, api, params, "u16", n, 1, 3, cap, srcs)
        got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, 1, 3, cap, srcs)
        assert got == want, cap


def test_arena_many_segments_per_frame(prod, eng, orc):
    """4 Mi-sample frames (256 segments: look-back chains of the cfg2 shape,
    the first round through scalar loads), one of them mixed."""
    rng = np.random.default_rng(3)
    n = 4 << 20
    params = api.CmpParams(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32,
                           checksum_enabled=1)
    srcs = [_signal(rng, n, "u16", "outliers"), _signal(rng, n, "u16", "mixed")]
    cap = 26 + 6 * n
    want = bs.run_batch_host(orc, api, params, "u16", n, 1, 2, cap, srcs)
    got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, 1, 2, cap, srcs)
    assert got == want
