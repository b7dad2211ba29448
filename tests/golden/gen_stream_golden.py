#!/usr/bin/env python3
"""Generate tests/golden/streams.json: payload-only streams (cmp_gpu_encode_stream)
as written by the REFERENCE's internal encoder API (oracle/ref_payload.c in
oracle/_ref/libref.so, compiled from /root/reference/lib).

Run from the repo root in the build container:
    make -C oracle ref && python3 tests/golden/gen_stream_golden.py

Inputs are the counter-hash synthetic frames of oracle/liborc.so
(orc_synth_u16 / orc_synth_i32), so a checker rebuilds them without the
reference.  Each case stores size and SHA-256 of the stream; the small cases
also store the stream bytes (hex).  The "cfg2_stream" case is BASELINE
configs[1] literally: ONE 64 Mi-sample 16-bit stream (the 16 cfg2 frames of
4 Mi samples, seed 0xA1A6, concatenated), DIFF + GOLOMB_ZERO g = 32.
"""
import ctypes
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "libref.so")
ORC = os.path.join(ROOT, "oracle", "liborc.so")

# (name, kind, pre, enc, g, outlier, seed, frames, n per frame, W)
CASES = [
    ("cfg2_stream", "u16", 1, 1, 32, 0, 0xA1A6, 16, 4 << 20, 32),
    ("u16_diff_zero_g5_1", "u16", 1, 1, 5, 0, 11, 1, 1, 32),
    ("u16_none_raw_1000", "u16", 0, 0, 1, 0, 12, 1, 1000, 32),
    ("u16_diff_multi_g8_o107", "u16", 1, 2, 8, 107, 13, 1, 70001, 32),
    ("u16_none_zero_g1_noise4096", "u16", 0, 1, 1, 0, 14, 1, 3 * 16384 + 5, 4096),
    ("u16_diff_zero_g1055", "u16", 1, 1, 1055, 0, 15, 1, 200000, 2048),
    ("i32_diff_zero_g16", "i16_in_i32", 1, 1, 16, 0, 16, 1, 5 * 8192 + 3, 32),
    ("i32_none_multi_g3_o9", "i16_in_i32", 0, 2, 3, 9, 17, 1, 40000, 8),
    ("u16_diff_zero_g32_1Mi", "u16", 1, 1, 32, 0, 18, 1, 1 << 20, 32),
]


def synth(orc, kind, seed, frames, n, W):
    if kind == "u16":
        x = np.empty(frames * n, dtype=np.uint16)
        for f in range(frames):
            orc.orc_synth_u16(seed, f, n, W, x[f * n:].ctypes.data)
    else:
        x = np.empty(frames * n, dtype=np.int32)
        for f in range(frames):
            orc.orc_synth_i32(seed, f, n, W, x[f * n:].ctypes.data)
    return x


def main():
    orc = ctypes.CDLL(ORC)
    ref = ctypes.CDLL(REF)
    for L in (orc,):
        L.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_void_p]
        L.orc_synth_i32.argtypes = L.orc_synth_u16.argtypes
    ref.ref_payload_stream.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p, ctypes.c_uint32]
    ref.ref_payload_stream.restype = ctypes.c_uint32
    out = {}
    for name, kind, pre, enc, g, outl, seed, frames, n, W in CASES:
        x = synth(orc, kind, seed, frames, n, W)
        N = frames * n
        cap = 6 * N + 64
        dst = np.zeros(cap + 8, dtype=np.uint8)
        off = (-dst.ctypes.data) % 8
        r = ref.ref_payload_stream(x.ctypes.data, N, 1 if kind != "u16" else 0, pre, enc, g, outl,
                                   dst.ctypes.data + off, cap)
        assert r < 0xFFFFFF00, (name, r)
        b = bytes(dst[off:off + r])
        d = dict(kind=kind, preprocessing=pre, encoder_type=enc, encoder_param=g, encoder_outlier=outl,
                 seed=seed, frames=frames, samples_per_frame=n, W=W, num_samples=N, size=r,
                 sha256=hashlib.sha256(b).hexdigest())
        if r <= 4096:
            d["hex"] = b.hex()
        out[name] = d
        print(name, N, r)
    with open(os.path.join(HERE, "streams.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_stream_golden.py",
                       reference="oracle/ref_payload.c + /root/reference/lib (oracle/_ref/libref.so)",
                       cases=out), f, indent=1)


if __name__ == "__main__":
    main()
