"""cmp_gpu_encode_stream (payload-only streams: one bit stream, no header, no
24-bit frame limit) against the reference's internal encoder path: the
golden streams of tests/golden/streams.json (written by the compiled
reference, oracle/ref_payload.c) -- BASELINE configs[1] literally, ONE
64 Mi-sample 16-bit stream with a single look-back chain of 4096 segments --
and the oracle's restatement on random inputs (every encoder, Rice and
general g, NONE/DIFF, both sample widths, whole and partial segments,
capacities that do not fit).  Bit-exact."""
import hashlib

import numpy as np
import pytest

import streams
from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


def gpu_stream(eng, x, kind, pre, enc, g, outl, cap=None):
    import torch
    n = x.size
    cap = 6 * n + 64 if cap is None else cap
    src = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).copy()).cuda()
    dst = torch.full(((cap + 64 + 7) // 8 * 8,), 0xAB, dtype=torch.uint8, device="cuda")
    size = torch.zeros(1, dtype=torch.int32, device="cuda")
    r = eng.encode_stream(kind, src.data_ptr(), n, pre, enc, g, outl, dst.data_ptr(), cap, size.data_ptr())
    if r:
        return r, b""
    assert eng.synchronize() == 0
    s = int(size.cpu().numpy().astype(np.uint32)[0])
    if api.is_error(s):
        return s, b""
    return s, bytes(dst[:s].cpu().numpy())


@pytest.mark.parametrize("name", sorted(streams.GOLD))
def test_stream_vs_reference_golden(eng, name):
    c = streams.GOLD[name]
    x = streams.synth(c)
    s, b = gpu_stream(eng, x, c["kind"], c["preprocessing"], c["encoder_type"], c["encoder_param"],
                      c["encoder_outlier"])
    assert s == c["size"], (s, c["size"])
    assert hashlib.sha256(b).hexdigest() == c["sha256"]


def test_stream_vs_oracle_random(eng):
    rng = np.random.default_rng(2024)
    bad = []
    seg16, seg32 = 4 * 4096, 2 * 4096
    for t in range(160):
        kind = ["u16", "i16", "i16_in_i32"][t % 3]
        seg = seg32 if kind == "i16_in_i32" else seg16
        n = int(rng.choice([rng.integers(1, 5000), rng.integers(1, 40) * seg,
                            rng.integers(1, 40) * seg + rng.integers(-30, 30), rng.integers(1, 400000)]))
        n = max(n, 1)
        pre, enc = int(rng.integers(0, 2)), int(rng.integers(0, 3))
        g = int(1 << rng.integers(0, 12)) if rng.random() < 0.5 else int(rng.integers(1, 3000))
        outl = int(rng.integers(1, 400))
        scale = 2.0 ** rng.uniform(0, 14)
        v = rng.laplace(0, scale, n)
        if rng.random() < 0.5:
            v = np.cumsum(v) * 0.05
        v = np.clip(np.round(v), -32768, 32767).astype(np.int64)
        if kind == "u16":
            x = (v & 0xFFFF).astype(np.uint16)
        elif kind == "i16":
            x = v.astype(np.int16)
        else:
            x = ((v & 0xFFFF) | (rng.integers(-9, 9, n) << 16)).astype(np.int32)
        want = streams.oracle_stream(x, kind, pre, enc, g, outl)
        got = gpu_stream(eng, x, kind, pre, enc, g, outl)
        if got != want:
            bad.append((t, kind, n, pre, enc, g, outl, got[0], want[0]))
    assert not bad, bad[:5]


def test_stream_capacity_and_arguments(eng):
    c = streams.GOLD["u16_diff_multi_g8_o107"]
    x = streams.synth(c)
    args = (c["kind"], c["preprocessing"], c["encoder_type"], c["encoder_param"], c["encoder_outlier"])
    s, _ = gpu_stream(eng, x, *args, cap=c["size"] - 1)
    assert api.error_name(s) == "DST_TOO_SMALL"
    s, b = gpu_stream(eng, x, *args, cap=c["size"])
    assert s == c["size"] and hashlib.sha256(b).hexdigest() == c["sha256"]
    # IWT / MODEL need a work buffer: not a stream mode
    assert api.error_name(gpu_stream(eng, x, c["kind"], 2, 1, 8, 0)[0]) == "PARAMS_INVALID"
    assert api.error_name(gpu_stream(eng, x, c["kind"], 3, 1, 8, 0)[0]) == "PARAMS_INVALID"
    assert api.error_name(gpu_stream(eng, x, c["kind"], 1, 1, 0, 0)[0]) == "PARAMS_INVALID"


@pytest.mark.parametrize("k", range(0, 8))
def test_stream_rice_kernel_vs_oracle(eng, k):
    """Streams the Rice/ZERO frame kernel takes (16-bit,
    GOLOMB_ZERO with g = 2^k, k <= 7, whole 16 Ki-sample segments, STREAM
    mode: no header, the first payload bit at 0): laplace noise at the scale
    of g, uniform noise (more bits than a segment's arena: chunk by chunk),
    1, 7 and 65 segments (the scalar look-back round past 16), NONE and DIFF,
    and a capacity one byte short."""
    rng = np.random.default_rng(300 + k)
    seg = 16384
    bad = []
    for m in (1, 7, 65):
        for data in ("laplace", "uniform"):
            n = m * seg
            if data == "laplace":
                v = np.round(rng.laplace(0, 2.0 ** k, n)).astype(np.int64)
                v = np.cumsum(v) if m == 7 else v
            else:
                v = rng.integers(-32768, 32768, n)
            kind = "u16" if (m + k) % 2 else "i16"
            x = (v & 0xFFFF).astype(np.uint16) if kind == "u16" else (v & 0xFFFF).astype(np.uint16).view(np.int16)
            for pre in (0, 1):
                want = streams.oracle_stream(x, kind, pre, 1, 1 << k, 0)
                got = gpu_stream(eng, x, kind, pre, 1, 1 << k, 0)
                if got != want:
                    bad.append((m, data, pre, got[0], want[0]))
    assert not bad, bad
    s, _ = gpu_stream(eng, x, kind, 1, 1, 1 << k, 0, cap=want[0] - 1)
    assert api.error_name(s) == "DST_TOO_SMALL"
