"""The oracle's payload-only stream (orc_payload_stream, the checker of
cmp_gpu_encode_stream) pinned to streams the REFERENCE wrote through its
internal encoder API (tests/golden/streams.json, oracle/ref_payload.c), and,
where oracle/_ref/libref.so is built, to that library directly on random
inputs.  CPU only."""
import ctypes
import hashlib

import numpy as np
import pytest

import streams
from conftest import REF_PATH


@pytest.mark.parametrize("name", sorted(streams.GOLD))
def test_oracle_stream_matches_reference_golden(name):
    c = streams.GOLD[name]
    x = streams.synth(c)
    r, b = streams.oracle_stream(x, c["kind"], c["preprocessing"], c["encoder_type"], c["encoder_param"],
                                 c["encoder_outlier"])
    assert r == c["size"]
    assert hashlib.sha256(b).hexdigest() == c["sha256"]
    if "hex" in c:
        assert b.hex() == c["hex"]


def test_oracle_stream_vs_compiled_reference_random():
    import os
    if not os.path.exists(REF_PATH):
        pytest.skip("oracle/_ref/libref.so not built (reference sources absent)")
    ref = ctypes.CDLL(REF_PATH, mode=ctypes.RTLD_LOCAL)
    ref.ref_payload_stream.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p, ctypes.c_uint32]
    ref.ref_payload_stream.restype = ctypes.c_uint32
    rng = np.random.default_rng(7)
    for t in range(300):
        kind = ["u16", "i16_in_i32"][t % 2]
        n = int(rng.integers(1, 3000))
        pre, enc = int(rng.integers(0, 2)), int(rng.integers(0, 3))
        g = int(rng.integers(1, 70)) if rng.random() < 0.8 else int(rng.integers(1, 65536))
        outl = int(rng.integers(1, 400))
        scale = 2.0 ** rng.uniform(0, 15)
        v = np.clip(np.round(rng.laplace(0, scale, n)), -32768, 32767).astype(np.int64)
        x = (v & 0xFFFF).astype(np.uint16) if kind == "u16" else ((v & 0xFFFF) | (rng.integers(0, 9, n) << 16)).astype(np.int32)
        cap = 6 * n + 64 if rng.random() < 0.8 else int(rng.integers(1, 6 * n + 64))
        r, b = streams.oracle_stream(x, kind, pre, enc, g, outl, cap)
        buf = np.zeros(cap + 8, dtype=np.uint8)
        off = (-buf.ctypes.data) % 8
        rr = ref.ref_payload_stream(x.ctypes.data, n, 0 if kind == "u16" else 1, pre, enc, g, outl,
                                    buf.ctypes.data + off, cap)
        assert r == rr, (t, r, rr)
        if rr < 0xFFFFFF00:
            assert b == bytes(buf[off:off + rr]), t
