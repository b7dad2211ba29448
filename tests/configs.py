"""BASELINE.json workloads as reproducible batches.

Inputs come from the counter-hash generator (oracle orc_synth_* on the CPU,
cmp_gpu_synthesize on the GPU; the two are checked equal in the GPU tests).
A config's digest is sha256 over its frames in index order with the header
identifier bytes 8..13 zeroed; sizes_digest is sha256 of the uint32 size array.
"""
import ctypes
import hashlib

import numpy as np

from conftest import load_pkg

api = load_pkg().cmpapi
P = api.CmpParams

DIFF, MODEL = 1, 3
ZERO, MULTI = 1, 2

CONFIGS = {
    # configs[0]: the example's parameters on 1 Ki samples, two acquisitions
    "cfg1_example": dict(kind="u16", n=1024, nctx=1, fpc=2, seed=0xA1A5, W=8,
                         params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO,
                                     primary_encoder_param=1055, secondary_iterations=15,
                                     secondary_preprocessing=MODEL, secondary_encoder_type=MULTI,
                                     secondary_encoder_param=8, secondary_encoder_outlier=107,
                                     model_rate=11, checksum_enabled=1, uncompressed_fallback_enabled=0)),
    # configs[1]: 64 Mi u16 samples, 16 frames of 4 Mi (24-bit size field), DIFF + ZERO g=32
    "cfg2_64Mi": dict(kind="u16", n=4 << 20, nctx=1, fpc=16, seed=0xA1A6, W=32,
                      params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO,
                                  primary_encoder_param=32)),
    # configs[2]: 1024 x 64 Ki, W_f = 2^(f mod 12), per-frame Rice k
    "cfg3_autorice": dict(kind="u16", n=64 << 10, nctx=1, fpc=1024, seed=0xA1A7, W="pow2_mod12",
                          auto_rice=True,
                          params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO,
                                      primary_encoder_param=32)),
    # configs[3]: 8192 x 64 Ki (frame f on GPU f mod 8), DIFF + ZERO g=32
    "cfg4_8192": dict(kind="u16", n=64 << 10, nctx=1, fpc=8192, seed=0xA1A8, W=32,
                      params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO,
                                  primary_encoder_param=32)),
    # configs[4]: 256 streams x 16 acquisitions x 64 Ki, i16 in i32, MODEL secondary
    "cfg5_model": dict(kind="i16_in_i32", n=64 << 10, nctx=256, fpc=16, seed=0xA1A9, W=32,
                       params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO,
                                   primary_encoder_param=16, secondary_iterations=15,
                                   secondary_preprocessing=MODEL, secondary_encoder_type=MULTI,
                                   secondary_encoder_param=8, secondary_encoder_outlier=107,
                                   model_rate=11)),
}


def noise_w(cfg, f):
    return (1 << (f % 12)) if cfg["W"] == "pow2_mod12" else cfg["W"]


def sample_bytes(cfg):
    return 4 if cfg["kind"] == "i16_in_i32" else 2


def gen_inputs_cpu(orc_ext, cfg, frames=None):
    """All frames (or the given frame indices) as a 2-D numpy array."""
    frames = range(cfg["nctx"] * cfg["fpc"]) if frames is None else frames
    frames = list(frames)
    n = cfg["n"]
    if sample_bytes(cfg) == 4:
        out = np.empty((len(frames), n), dtype=np.int32)
        for i, f in enumerate(frames):
            orc_ext.orc_synth_i32(cfg["seed"], f, n, noise_w(cfg, f), out[i].ctypes.data)
    else:
        out = np.empty((len(frames), n), dtype=np.uint16)
        for i, f in enumerate(frames):
            orc_ext.orc_synth_u16(cfg["seed"], f, n, noise_w(cfg, f), out[i].ctypes.data)
    return out


def frame_digest(frames_bytes):
    """frames_bytes: iterable of bytes objects, one per frame, in order."""
    h = hashlib.sha256()
    sizes = []
    for b in frames_bytes:
        b = bytearray(b)
        b[8:14] = b"\0" * 6
        h.update(b)
        sizes.append(len(b))
    return dict(digest=h.hexdigest(), total_bytes=int(sum(sizes)),
                sizes_digest=hashlib.sha256(np.array(sizes, dtype=np.uint32).tobytes()).hexdigest())


def rice_ks(orc_ext, cfg, data):
    ks = []
    for i in range(data.shape[0]):
        ks.append(orc_ext.orc_select_rice_k(data[i].ctypes.data, cfg["n"], 1 if sample_bytes(cfg) == 4 else 0,
                                            cfg["params"]["primary_preprocessing"], None))
    return ks


def cpu_frames(lib_path, orc_ext, cfg, threads=8):
    """Run a config through a CPU implementation of cmp.h (oracle or reference).

    Returns (list of frame bytes, list of rice g or None)."""
    lib = api.CmpLib(lib_path)
    data = gen_inputs_cpu(orc_ext, cfg)
    nframes = data.shape[0]
    n, sb = cfg["n"], sample_bytes(cfg)
    bound = lib.compress_bound(2 * n)
    cap = bound if not api.is_error(bound) else (2 * n * 3 + 64)
    stride = (cap + 7) // 8 * 8
    dst = api.aligned_empty(stride * nframes)
    sizes = np.zeros(nframes, dtype=np.uint32)
    gs = None
    if cfg.get("auto_rice"):
        ks = rice_ks(orc_ext, cfg, data)
        gs = [1 << k for k in ks]
        for f in range(nframes):
            prm = P(**dict(cfg["params"], primary_encoder_param=gs[f]))
            ctx = api.CmpContext()
            assert not api.is_error(lib.initialise(ctx, prm))
            r = lib.compress(cfg["kind"], ctx, dst[f * stride:], cap, data[f])
            assert not api.is_error(r), api.error_name(r)
            sizes[f] = r
    else:
        drv = ctypes.CDLL(lib_path, mode=ctypes.RTLD_LOCAL)
        drv.drv_run.restype = ctypes.c_uint64
        prm = P(**cfg["params"])
        tot = drv.drv_run(ctypes.byref(prm), {"u16": 0, "i16": 1, "i16_in_i32": 2}[cfg["kind"]],
                          ctypes.c_void_p(data.ctypes.data), ctypes.c_uint32(n * sb), ctypes.c_uint64(n * sb),
                          ctypes.c_uint32(cfg["nctx"]), ctypes.c_uint32(cfg["fpc"]),
                          ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                          ctypes.c_void_p(sizes.ctypes.data), ctypes.c_int(threads), ctypes.c_int(1))
        assert tot != 2**64 - 1, "drv_run failed"
    frames = [bytes(dst[f * stride:f * stride + int(sizes[f])]) for f in range(nframes)]
    return frames, gs


def reference_digest(name, lib_path):
    import conftest
    orc_ext = ctypes.CDLL(conftest.ORC_PATH, mode=ctypes.RTLD_LOCAL)
    orc_ext.orc_select_rice_k.restype = ctypes.c_uint32
    orc_ext.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_void_p]
    orc_ext.orc_synth_i32.argtypes = orc_ext.orc_synth_u16.argtypes
    orc_ext.orc_select_rice_k.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]
    frames, gs = cpu_frames(lib_path, orc_ext, CONFIGS[name])
    d = frame_digest(frames)
    if name == "cfg4_8192":
        # bench.py shards: rank r of N encodes frames r + N*j, j < 1024
        for nw in (1, 2, 4, 8):
            d[f"shard_digests_n{nw}"] = [frame_digest(frames[r::nw][:1024])["digest"] for r in range(nw)]
            # what rank 0 holds after gathering N shards: frames 0 .. 1024*N-1 in f order
            d[f"gather_digest_n{nw}"] = frame_digest(frames[:1024 * nw])["digest"]
    if name == "cfg5_model":
        # streams sharded s mod N (bench.py cfg5 shard workloads): rank r of N
        # holds streams r, r + N, ..., each stream's 16 frames in order
        fpc, ns = CONFIGS[name]["fpc"], CONFIGS[name]["nctx"]
        for nw in (2, 4, 8):
            d[f"shard_digests_n{nw}"] = [frame_digest([frames[s * fpc + a] for s in range(r, ns, nw)
                                                       for a in range(fpc)])["digest"] for r in range(nw)]
    if gs is not None:
        d["rice_g_digest"] = hashlib.sha256(np.array(gs, dtype=np.uint32).tobytes()).hexdigest()
    return d


def gpu_frames(lib, eng, cfg, return_model=False):
    """Run a config through the GPU batch API (cmp_gpu_compress); returns
    (frame bytes list, per-frame g or None, sizes array)."""
    import torch
    n, sb = cfg["n"], sample_bytes(cfg)
    nctx, fpc = cfg["nctx"], cfg["fpc"]
    nframes = nctx * fpc
    stride = n * sb
    src = torch.empty(nframes * stride, dtype=torch.uint8, device="cuda")
    if cfg["W"] == "pow2_mod12":
        for f in range(nframes):
            assert eng.synthesize(src.data_ptr() + f * stride, sb, cfg["seed"], f, n, 1, stride,
                                  noise_w(cfg, f)) == 0
    else:
        assert eng.synthesize(src.data_ptr(), sb, cfg["seed"], 0, n, nframes, stride, cfg["W"]) == 0
    bound = lib.compress_bound(2 * n)
    cap = bound if not api.is_error(bound) else (2 * n * 3 + 64)
    dstride = (cap + 7) // 8 * 8
    dst = torch.empty(nframes * dstride, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nframes, dtype=torch.int32, device="cuda")
    prm = P(**cfg["params"])
    wbs = lib.cal_work_buf_size(prm, stride)
    wstride = (wbs + 15) // 16 * 16
    work = torch.zeros(max(nctx * wstride, 16), dtype=torch.uint8, device="cuda")
    ctxs = (api.CmpContext * nctx)()
    for c in range(nctx):
        r = lib.initialise(ctxs[c], prm, (work.data_ptr() + c * wstride) if wbs else None, wbs)
        assert not api.is_error(r), api.error_name(r)
    flags = 1 if cfg.get("auto_rice") else 0
    torch.cuda.synchronize()
    r = eng.compress(ctxs, fpc, cfg["kind"], src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                     sizes.data_ptr(), flags)
    assert r == 0, api.error_name(r)
    assert eng.synchronize() == 0
    sz = sizes.cpu().numpy().astype(np.uint32)
    assert not any(api.is_error(int(s)) for s in sz), [api.error_name(int(s)) for s in sz[:4]]
    host = dst.cpu().numpy()
    frames = [bytes(host[f * dstride:f * dstride + int(sz[f])]) for f in range(nframes)]
    gs = None
    if cfg.get("auto_rice"):
        gs = [api.parse_header(fr)["encoder_param"] for fr in frames]
    if return_model:
        return frames, gs, sz, work.cpu().numpy(), wstride
    return frames, gs, sz
