"""Shared helpers for the payload-only stream tests (cmp_gpu_encode_stream):
golden cases (tests/golden/streams.json, made by gen_stream_golden.py from
the reference's internal encoder API) and the oracle's restatement."""
import ctypes
import json
import os

import numpy as np

from conftest import GOLDEN_DIR, ORC_PATH

with open(os.path.join(GOLDEN_DIR, "streams.json")) as _f:
    GOLD = json.load(_f)["cases"]

_orc = None


def orc():
    global _orc
    if _orc is None:
        L = ctypes.CDLL(ORC_PATH, mode=ctypes.RTLD_LOCAL)
        L.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_void_p]
        L.orc_synth_i32.argtypes = L.orc_synth_u16.argtypes
        L.orc_payload_stream.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p, ctypes.c_uint32]
        L.orc_payload_stream.restype = ctypes.c_uint32
        _orc = L
    return _orc


def synth(case):
    L = orc()
    n, frames = case["samples_per_frame"], case["frames"]
    if case["kind"] == "u16":
        x = np.empty(frames * n, dtype=np.uint16)
        fn = L.orc_synth_u16
    else:
        x = np.empty(frames * n, dtype=np.int32)
        fn = L.orc_synth_i32
    for f in range(frames):
        fn(case["seed"], f, n, case["W"], x[f * n:].ctypes.data)
    return x


def oracle_stream(x, kind, pre, enc, g, outlier, cap=None):
    """(size or error value, bytes) of the oracle's payload-only stream."""
    N = x.size
    cap = 6 * N + 64 if cap is None else cap
    buf = np.zeros(cap + 8, dtype=np.uint8)
    off = (-buf.ctypes.data) % 8
    r = orc().orc_payload_stream(np.ascontiguousarray(x).ctypes.data, N, 0 if kind in ("u16", "i16") else 1,
                                 pre, enc, g, outlier, buf.ctypes.data + off, cap)
    return r, bytes(buf[off:off + r]) if r < 0xFFFFFF00 else b""
