"""ctypes mirror of the cmp.h compression API.

One wrapper class drives any shared library that exports the reference's
lib/cmp.h + lib/cmp_errors.h symbols (the MI355X product library
``lib/libairscmp.so``; the test suite also points it at its CPU checkers).
Struct layouts mirror reference lib/cmp.h:94-137 (cmp_params 44 B,
cmp_context 80 B on x86-64); enum values mirror lib/cmp.h:64-82 and
lib/cmp_errors.h:28-60.
"""
from __future__ import annotations

import ctypes
from ctypes import c_int, c_uint8, c_uint32, c_uint64, c_void_p, c_char_p, POINTER

import numpy as np

# enum cmp_preprocessing (reference lib/cmp.h:64-71)
PREPROCESS_NONE, PREPROCESS_DIFF, PREPROCESS_IWT, PREPROCESS_MODEL = range(4)
# enum cmp_encoder_type (reference lib/cmp.h:78-82)
ENCODER_UNCOMPRESSED, ENCODER_GOLOMB_ZERO, ENCODER_GOLOMB_MULTI = range(3)

# enum cmp_error (reference lib/cmp_errors.h:28-60)
ERR = dict(
    NO_ERROR=0, GENERIC=1, PARAMS_INVALID=10, DST_TOO_SMALL=30, DST_NULL=31,
    DST_UNALIGNED=32, SRC_SIZE_WRONG=40, SRC_NULL=41, SRC_SIZE_MISMATCH=42,
    WORK_BUF_TOO_SMALL=50, WORK_BUF_NULL=51, WORK_BUF_UNALIGNED=52,
    HDR_CMP_SIZE_TOO_LARGE=60, HDR_ORIGINAL_TOO_LARGE=61, CONTEXT_INVALID=70,
    INT_HDR=100, INT_ENCODER=101, INT_BITSTREAM=102, MAX_CODE=128,
)

CMP_HDR_SIZE = 16
CMP_HDR_MAX_SIZE = 22
CMP_CHECKSUM_SIZE = 4
CMP_HDR_MAX_COMPRESSED_SIZE = (1 << 24) - 1
CMP_HDR_MAX_ORIGINAL_SIZE = (1 << 24) - 1
CMP_VERSION_NUMBER = 600
# cmp_gpu_batch.flags (include/cmp_gpu.h)
GPU_AUTO_RICE = 0x1
GPU_HOST_STEPPED = 0x2
GPU_STEPWISE = 0x4
GPU_REPORT_DRAWS = 0x8


def err_value(name: str) -> int:
    """(uint32_t)-code, the value the API returns for an error."""
    return (-ERR[name]) & 0xFFFFFFFF


def is_error(v: int) -> bool:
    return (v & 0xFFFFFFFF) > err_value("MAX_CODE")


def error_code(v: int) -> int:
    return ((-v) & 0xFFFFFFFF) if is_error(v) else 0


def error_name(v: int) -> str:
    c = error_code(v)
    for k, x in ERR.items():
        if x == c:
            return k
    return str(c)


def uncompressed_bound(packed_size: int) -> int:
    """CMP_UNCOMPRESSED_BOUND (reference lib/cmp.h:212-215)."""
    if packed_size <= CMP_HDR_MAX_COMPRESSED_SIZE - CMP_HDR_SIZE - CMP_CHECKSUM_SIZE:
        return CMP_HDR_SIZE + packed_size + CMP_CHECKSUM_SIZE
    return 2**64 - 1


class CmpParams(ctypes.Structure):
    _fields_ = [
        ("primary_preprocessing", c_int),
        ("primary_encoder_type", c_int),
        ("primary_encoder_param", c_uint32),
        ("primary_encoder_outlier", c_uint32),
        ("secondary_iterations", c_uint32),
        ("secondary_preprocessing", c_int),
        ("secondary_encoder_type", c_int),
        ("secondary_encoder_param", c_uint32),
        ("secondary_encoder_outlier", c_uint32),
        ("model_rate", c_uint32),
        ("checksum_enabled", c_uint8),
        ("uncompressed_fallback_enabled", c_uint8),
    ]

    def __init__(self, **kw):
        super().__init__()
        for k, v in kw.items():
            setattr(self, k, v)

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class CmpContext(ctypes.Structure):
    _fields_ = [
        ("magic", c_uint32),
        ("params", CmpParams),
        ("work_buf", c_void_p),
        ("work_buf_size", c_uint32),
        ("model_size", c_uint32),
        ("identifier", c_uint64),
        ("sequence_number", c_uint8),
    ]


assert ctypes.sizeof(CmpParams) == 44
assert ctypes.sizeof(CmpContext) == 80

TIMESTAMP_FN = ctypes.CFUNCTYPE(None, POINTER(c_uint32), POINTER(ctypes.c_uint16))

# the C-ABI symbols every implementation exports (include/cmp.h, cmp_errors.h)
API_SYMBOLS = (
    "cmp_set_timestamp_func", "cmp_is_error", "cmp_compress_bound", "cmp_cal_work_buf_size",
    "cmp_initialise", "cmp_compress_i16", "cmp_compress_i16_in_i32", "cmp_compress_u16",
    "cmp_reset", "cmp_deinitialise", "cmp_get_error_code", "cmp_get_error_message",
    "cmp_get_error_string",
)


def aligned_empty(nbytes: int, align: int = 64, fill: int | None = None) -> np.ndarray:
    """uint8 array whose data pointer is `align`-byte aligned (dst must be 8-aligned)."""
    raw = np.empty(nbytes + align, dtype=np.uint8)
    off = (-raw.ctypes.data) % align
    a = raw[off:off + nbytes]
    if fill is not None:
        a[:] = fill
    return a


class CmpLib:
    """Thin ctypes wrapper; method names follow lib/cmp.h without the prefix."""

    def __init__(self, path: str):
        self.path = path
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        L = self.lib
        L.cmp_set_timestamp_func.argtypes = [TIMESTAMP_FN]
        L.cmp_set_timestamp_func.restype = None
        L.cmp_is_error.argtypes = [c_uint32]
        L.cmp_is_error.restype = ctypes.c_uint
        L.cmp_compress_bound.argtypes = [c_uint32]
        L.cmp_compress_bound.restype = c_uint32
        L.cmp_cal_work_buf_size.argtypes = [POINTER(CmpParams), c_uint32]
        L.cmp_cal_work_buf_size.restype = c_uint32
        L.cmp_initialise.argtypes = [POINTER(CmpContext), POINTER(CmpParams), c_void_p, c_uint32]
        L.cmp_initialise.restype = c_uint32
        for n in ("cmp_compress_u16", "cmp_compress_i16", "cmp_compress_i16_in_i32"):
            f = getattr(L, n)
            f.argtypes = [POINTER(CmpContext), c_void_p, c_uint32, c_void_p, c_uint32]
            f.restype = c_uint32
        L.cmp_reset.argtypes = [POINTER(CmpContext)]
        L.cmp_reset.restype = c_uint32
        L.cmp_deinitialise.argtypes = [POINTER(CmpContext)]
        L.cmp_deinitialise.restype = None
        L.cmp_get_error_code.argtypes = [c_uint32]
        L.cmp_get_error_code.restype = c_int
        L.cmp_get_error_message.argtypes = [c_uint32]
        L.cmp_get_error_message.restype = c_char_p
        L.cmp_get_error_string.argtypes = [c_int]
        L.cmp_get_error_string.restype = c_char_p
        self._ts_keepalive = None

    # -- API -------------------------------------------------------------
    def set_timestamp_func(self, fn):
        """fn() -> (coarse, fine) or None to restore the built-in counter."""
        if fn is None:
            self._ts_keepalive = None
            self.lib.cmp_set_timestamp_func(ctypes.cast(None, TIMESTAMP_FN))
            return

        def _cb(pc, pf):
            c, f = fn()
            pc[0] = c & 0xFFFFFFFF
            pf[0] = f & 0xFFFF

        self._ts_keepalive = TIMESTAMP_FN(_cb)
        self.lib.cmp_set_timestamp_func(self._ts_keepalive)

    def is_error(self, v):
        return bool(self.lib.cmp_is_error(v & 0xFFFFFFFF))

    def compress_bound(self, packed_size):
        return self.lib.cmp_compress_bound(packed_size)

    def cal_work_buf_size(self, params, src_size):
        return self.lib.cmp_cal_work_buf_size(None if params is None else ctypes.byref(params), src_size)

    def initialise(self, ctx, params, work_buf=None, work_buf_size=0):
        wb = work_buf if (work_buf is None or isinstance(work_buf, int)) else work_buf.ctypes.data
        return self.lib.cmp_initialise(None if ctx is None else ctypes.byref(ctx),
                                       None if params is None else ctypes.byref(params),
                                       wb, work_buf_size & 0xFFFFFFFF)

    def _compress(self, fn, ctx, dst, cap, src, src_size):
        d = dst if (dst is None or isinstance(dst, int)) else dst.ctypes.data
        s = src if (src is None or isinstance(src, int)) else src.ctypes.data
        if src_size is None:
            src_size = src.nbytes
        return fn(None if ctx is None else ctypes.byref(ctx), d, cap & 0xFFFFFFFF, s, src_size & 0xFFFFFFFF)

    def compress_u16(self, ctx, dst, cap, src, src_size=None):
        return self._compress(self.lib.cmp_compress_u16, ctx, dst, cap, src, src_size)

    def compress_i16(self, ctx, dst, cap, src, src_size=None):
        return self._compress(self.lib.cmp_compress_i16, ctx, dst, cap, src, src_size)

    def compress_i16_in_i32(self, ctx, dst, cap, src, src_size=None):
        return self._compress(self.lib.cmp_compress_i16_in_i32, ctx, dst, cap, src, src_size)

    def compress(self, kind, ctx, dst, cap, src, src_size=None):
        f = {"u16": self.compress_u16, "i16": self.compress_i16, "i16_in_i32": self.compress_i16_in_i32}[kind]
        return f(ctx, dst, cap, src, src_size)

    def reset(self, ctx):
        return self.lib.cmp_reset(None if ctx is None else ctypes.byref(ctx))

    def deinitialise(self, ctx):
        self.lib.cmp_deinitialise(None if ctx is None else ctypes.byref(ctx))

    def get_error_code(self, v):
        return self.lib.cmp_get_error_code(v & 0xFFFFFFFF)

    def get_error_message(self, v):
        return self.lib.cmp_get_error_message(v & 0xFFFFFFFF).decode()

    def get_error_string(self, code):
        return self.lib.cmp_get_error_string(code).decode()


def parse_header(buf) -> dict:
    """Decode a frame header (format of reference lib/common/header.c:89-134)."""
    b = bytes(buf[:22])
    h = dict(
        version_flag=b[0] >> 7,
        version_id=((b[0] & 0x7F) << 8) | b[1],
        compressed_size=int.from_bytes(b[2:5], "big"),
        original_size=int.from_bytes(b[5:8], "big"),
        identifier=int.from_bytes(b[8:14], "big"),
        sequence_number=b[14],
        preprocessing=b[15] >> 4,
        checksum_enabled=(b[15] >> 3) & 1,
        encoder_type=b[15] & 7,
        model_rate=0, encoder_param=0, encoder_outlier=0,
    )
    if not (h["preprocessing"] == PREPROCESS_NONE and h["encoder_type"] == ENCODER_UNCOMPRESSED):
        h["model_rate"] = b[16]
        h["encoder_param"] = int.from_bytes(b[17:19], "big")
        h["encoder_outlier"] = int.from_bytes(b[19:22], "big")
        h["header_size"] = 22
    else:
        h["header_size"] = 16
    return h
