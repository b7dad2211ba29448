"""airs-compression_amd -- MI355X-native AIRSPACE encode path.

Python side of the drop-in: ctypes bindings over ``lib/libairscmp.so``
(built from ``csrc/`` by the Makefile).  ``cmpapi`` mirrors the reference's
lib/cmp.h API; :class:`GpuEngine` binds the device batch API of
include/cmp_gpu.h.  The library has no CPU encode path: compress calls need
the HIP device, and loading fails loudly when the shared object is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_uint32, c_uint64, c_void_p

from .cmpapi import *  # noqa: F401,F403
from .cmpapi import CmpContext, CmpLib, is_error, error_name

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libairscmp.so")

GPU_U16, GPU_I16, GPU_I16_IN_I32 = 0, 1, 2
GPU_AUTO_RICE = 0x1
REPORT_DRAWS = 0x8  # CMP_GPU_REPORT_DRAWS
LAYOUT_ROUNDROBIN, LAYOUT_BLOCK, LAYOUT_STREAMS = 0, 1, 2  # enum cmp_gpu_layout
GATHER_PATCH_IDS = 0x1  # CMP_GPU_GATHER_PATCH_IDS
OPT_EXCLUSIVE = 1  # cmp_gpu_engine_set_option (include/cmp_gpu.h)
OPT_WALK_SEGMENT = 2
OPT_NO_CONTEXT_WALK = 3
KIND_TO_GPU = {"u16": GPU_U16, "i16": GPU_I16, "i16_in_i32": GPU_I16_IN_I32}


def build(jobs: int = 8) -> str:
    """Compile csrc/ into lib/libairscmp.so (hipcc for gfx950 + gcc)."""
    subprocess.run(["make", f"-j{jobs}", "-C", PKG_DIR], check=True)
    return LIB_PATH


def _one_hip_runtime() -> None:
    """PyTorch-ROCm ships its own libamdhip64.so (SONAME libamdhip64.so.7, the
    same as /opt/rocm's).  If libairscmp.so were dlopen'ed first, torch would
    later map a second HIP runtime into the process and fail to see the GPU.
    Importing torch first makes the library bind to torch's copy, so device
    pointers, streams and events are shared.  Without torch the library uses
    /opt/rocm's runtime as usual."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load(path: str | None = None) -> "AirsLib":
    # AIRS_LIB: developer override (benchmarking an alternative build)
    path = path or os.environ.get("AIRS_LIB") or LIB_PATH
    _one_hip_runtime()
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} is missing: build it with `make -C {PKG_DIR}` (no CPU fallback exists)")
    return AirsLib(path)


class GpuBatch(ctypes.Structure):
    """struct cmp_gpu_batch (include/cmp_gpu.h)."""
    _fields_ = [
        ("type", c_int),
        ("src", c_void_p),
        ("src_stride", c_uint64),
        ("src_size", c_uint32),
        ("dst", c_void_p),
        ("dst_stride", c_uint64),
        ("dst_capacity", c_uint32),
        ("sizes", c_void_p),
        ("flags", c_uint32),
        ("draws", c_void_p),
    ]


class GpuDecodeBatch(ctypes.Structure):
    """struct cmp_gpu_decode_batch (include/cmp_gpu.h)."""
    _fields_ = [
        ("src", c_void_p),
        ("src_stride", c_uint64),
        ("src_capacity", c_uint32),
        ("num_frames", c_uint32),
        ("dst", c_void_p),
        ("dst_stride", c_uint64),
        ("dst_samples", c_uint32),
        ("status", c_void_p),
        ("model", c_void_p),
        ("model_stride", c_uint64),
    ]


class AirsLib(CmpLib):
    """CmpLib plus the cmp_gpu.h device batch API."""

    def __init__(self, path: str = LIB_PATH):
        super().__init__(path)
        L = self.lib
        L.cmp_gpu_available.restype = c_int
        L.cmp_gpu_engine_create.argtypes = [POINTER(c_void_p), c_void_p]
        L.cmp_gpu_engine_create.restype = c_uint32
        L.cmp_gpu_engine_destroy.argtypes = [c_void_p]
        L.cmp_gpu_engine_destroy.restype = None
        L.cmp_gpu_engine_set_option.argtypes = [c_void_p, c_uint32, c_uint32]
        L.cmp_gpu_engine_set_option.restype = c_uint32
        L.cmp_gpu_compress.argtypes = [c_void_p, POINTER(CmpContext), c_uint32, c_uint32, POINTER(GpuBatch)]
        L.cmp_gpu_compress.restype = c_uint32
        L.cmp_gpu_synchronize.argtypes = [c_void_p]
        L.cmp_gpu_synchronize.restype = c_uint32
        L.cmp_gpu_synthesize.argtypes = [c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_uint32,
                                         c_uint32, c_uint64, c_uint32]
        L.cmp_gpu_synthesize.restype = c_uint32
        L.cmp_gpu_decompress.argtypes = [c_void_p, POINTER(GpuDecodeBatch)]
        L.cmp_gpu_decompress.restype = c_uint32
        L.cmp_gpu_encode_stream.argtypes = [c_void_p, c_uint32, c_void_p, c_uint32, c_uint32, c_uint32, c_uint32,
                                            c_uint32, c_void_p, c_uint32, c_void_p]
        L.cmp_gpu_encode_stream.restype = c_uint32
        L.cmp_gpu_pack_frames.argtypes = [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint32, c_void_p,
                                          c_void_p]
        L.cmp_gpu_pack_frames.restype = c_uint32
        L.cmp_gpu_gather.argtypes = [c_void_p, c_void_p, c_uint32, c_uint32, c_uint32, c_void_p, c_uint64, c_uint32,
                                     c_void_p, c_void_p, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64,
                                     c_uint32]
        L.cmp_gpu_gather.restype = c_uint32
        L.cmp_gpu_gather_plan.argtypes = [c_void_p, c_uint32, c_uint32, c_uint32, c_uint32, c_uint64, c_void_p,
                                          c_void_p, c_void_p, c_void_p]
        L.cmp_gpu_gather_plan.restype = c_uint32

    def gpu_available(self) -> bool:
        return bool(self.lib.cmp_gpu_available())

    def gather_plan(self, entries, world: int, frames_per_rank: int, layout: int, fpc: int = 1,
                    id_base: int = 0, want_ids: bool = True):
        """cmp_gpu_gather_plan on host arrays (no device): entries uint64
        [world * frames_per_rank] = size | draws << 32.  Returns (rc,
        rank_bytes, offsets, sizes, ids or None), the last three in global
        frame order; ids UINT64_MAX where a frame keeps its identifier."""
        import numpy as np
        e = np.ascontiguousarray(entries, dtype=np.uint64)
        n = world * frames_per_rank
        rb = np.zeros(world, dtype=np.uint64)
        offs = np.zeros(max(n, 1), dtype=np.uint64)
        sz = np.zeros(max(n, 1), dtype=np.uint32)
        ids = np.zeros(max(n, 1), dtype=np.uint64) if want_ids else None
        r = self.lib.cmp_gpu_gather_plan(e.ctypes.data, world, frames_per_rank, layout, fpc, id_base, rb.ctypes.data,
                                         offs.ctypes.data, sz.ctypes.data, ids.ctypes.data if want_ids else None)
        return int(r), rb, offs[:n], sz[:n], (ids[:n] if want_ids else None)

    def engine(self, stream: int | None = None) -> "GpuEngine":
        return GpuEngine(self, stream)


class GpuEngine:
    """One cmp_gpu_engine bound to a HIP stream (raw hipStream_t handle)."""

    def __init__(self, lib: AirsLib, stream: int | None = None):
        self.lib = lib
        self.stream = stream  # raw hipStream_t the engine's work is queued on (None: the null stream)
        h = c_void_p()
        r = lib.lib.cmp_gpu_engine_create(ctypes.byref(h), stream)
        if is_error(r):
            raise RuntimeError(f"cmp_gpu_engine_create failed: {error_name(r)}")
        self.handle = h

    def set_option(self, option: int, value: int) -> int:
        """cmp_gpu_engine_set_option (OPT_EXCLUSIVE, OPT_WALK_SEGMENT, OPT_NO_CONTEXT_WALK)."""
        return int(self.lib.lib.cmp_gpu_engine_set_option(self.handle, option, value))

    def close(self):
        if self.handle:
            self.lib.lib.cmp_gpu_engine_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress(self, ctxs, frames_per_ctx: int, kind: str, src_ptr: int, src_stride: int,
                 src_size: int, dst_ptr: int, dst_stride: int, dst_capacity: int, sizes_ptr: int,
                 flags: int = 0, draws_ptr: int | None = None) -> int:
        """cmp_gpu_compress over device pointers; ctxs is a ctypes CmpContext array.
        draws_ptr: optional host uint8 array receiving each frame's identifier draws."""
        if draws_ptr:
            flags |= REPORT_DRAWS
        b = GpuBatch(type=KIND_TO_GPU[kind], src=src_ptr, src_stride=src_stride, src_size=src_size,
                     dst=dst_ptr, dst_stride=dst_stride, dst_capacity=dst_capacity,
                     sizes=sizes_ptr, flags=flags, draws=draws_ptr)
        n_ctx = len(ctxs)
        return self.lib.lib.cmp_gpu_compress(self.handle, ctxs, n_ctx, frames_per_ctx, ctypes.byref(b))

    def decompress(self, src_ptr: int, src_stride: int, src_capacity: int, num_frames: int, dst_ptr: int,
                   dst_stride: int, dst_samples: int, status_ptr: int, model_ptr: int = 0,
                   model_stride: int = 0) -> int:
        """cmp_gpu_decompress over device pointers (frames -> 16-bit samples)."""
        b = GpuDecodeBatch(src=src_ptr, src_stride=src_stride, src_capacity=src_capacity, num_frames=num_frames,
                           dst=dst_ptr, dst_stride=dst_stride, dst_samples=dst_samples, status=status_ptr,
                           model=model_ptr or None, model_stride=model_stride)
        return self.lib.lib.cmp_gpu_decompress(self.handle, ctypes.byref(b))

    def encode_stream(self, kind: str, src_ptr: int, num_samples: int, preprocessing: int, encoder_type: int,
                      encoder_param: int, encoder_outlier: int, dst_ptr: int, dst_capacity: int,
                      size_ptr: int) -> int:
        """cmp_gpu_encode_stream: one payload-only bit stream (no header) over device pointers."""
        return self.lib.lib.cmp_gpu_encode_stream(self.handle, KIND_TO_GPU[kind], src_ptr, num_samples,
                                                  preprocessing, encoder_type, encoder_param, encoder_outlier,
                                                  dst_ptr, dst_capacity, size_ptr)

    def pack_frames(self, frames_ptr: int, frame_stride: int, frame_capacity: int, sizes_ptr: int,
                    num_frames: int, out_ptr: int, offsets_ptr: int) -> int:
        """cmp_gpu_pack_frames: strided frames -> back to back at 8-byte aligned offsets (device)."""
        return self.lib.lib.cmp_gpu_pack_frames(self.handle, frames_ptr, frame_stride, frame_capacity, sizes_ptr,
                                                num_frames, out_ptr, offsets_ptr)

    def gather(self, nccl_comm: int, root: int, layout: int, fpc: int, frames_ptr: int, frame_stride: int,
               frame_capacity: int, sizes_ptr: int, draws_ptr: int | None, frames_per_rank: int, out_ptr: int | None,
               out_capacity: int, offsets_ptr: int | None, out_sizes_ptr: int | None, id_base: int = 0,
               flags: int = 0) -> int:
        """cmp_gpu_gather: every rank's frames on `root` over an RCCL communicator (ncclComm_t as an int)."""
        return self.lib.lib.cmp_gpu_gather(self.handle, nccl_comm, root, layout, fpc, frames_ptr, frame_stride,
                                           frame_capacity, sizes_ptr, draws_ptr, frames_per_rank, out_ptr,
                                           out_capacity, offsets_ptr, out_sizes_ptr, id_base, flags)

    def synchronize(self) -> int:
        return self.lib.lib.cmp_gpu_synchronize(self.handle)

    def synthesize(self, dst_ptr: int, sample_bytes: int, seed: int, frame0: int, n: int,
                   num_frames: int, stride: int, noise_w: int) -> int:
        return self.lib.lib.cmp_gpu_synthesize(self.handle, dst_ptr, sample_bytes, seed, frame0, n,
                                               num_frames, stride, noise_w)


def context_array(n: int):
    return (CmpContext * n)()


def __getattr__(name):
    # submodules that need torch are imported on first use
    if name == "shard":
        import importlib
        return importlib.import_module(__name__ + ".shard")
    raise AttributeError(name)
