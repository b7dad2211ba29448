"""Batch-API scenarios: cmp_gpu_compress against the c-major loop of
cmp_compress_* calls it is defined to equal (include/cmp_gpu.h).

`run_batch_host` runs any CmpLib (the oracle) frame by frame in call order;
`run_batch_gpu` runs the same frames through one cmp_gpu_compress call on
device buffers.  Both return the same observable tuple: per frame the return
value and bytes, per context identifier / sequence number / model size and
the work buffer (model).
"""
import random

import numpy as np

import scenarios


def _ts_counter(start):
    stamp = [start]

    def ts():
        stamp[0] += 1
        return (stamp[0] >> 16, stamp[0] & 0xFFFF)
    return ts


def make_case(api, trial):
    """Seeded batch case: params, kind, n, nctx, fpc, cap, per-frame sources."""
    rng = random.Random(trial)
    params = scenarios.make_params(api.CmpParams, rng, allow_iwt=True)
    params.uncompressed_fallback_enabled = rng.choice([0, 1, 1])
    kind = rng.choice(scenarios.KINDS)
    n = rng.choice([1, 7, 64, 333, 4095, 4097, 9000])
    nctx = rng.choice([1, 2, 3])
    fpc = rng.choice([1, 3, 6])
    raw = 16 + 2 * n + (4 if params.checksum_enabled else 0)
    worst = 22 + 4 + 6 * n
    cap = rng.choice([worst, raw, raw + 3, raw - 1, 22 + n, 40])
    srcs = [scenarios.make_src(kind, n, rng, rng.choice([1, 50, 3000, 30000])) for _ in range(nctx * fpc)]
    return params, kind, n, nctx, fpc, cap, srcs


def _work_size(lib, api, params, nbytes):
    w = lib.cal_work_buf_size(params, nbytes)
    return 0 if api.is_error(w) else w


def _per_ctx(params, nctx):
    """one params for every context, or a list of per-context params"""
    return list(params) if isinstance(params, (list, tuple)) else [params] * nctx


def _calls(fpc, splits):
    """(first acquisition, acquisitions) of each cmp_gpu_compress call"""
    splits = list(splits) if splits else [fpc]
    assert sum(splits) == fpc
    out, a0 = [], 0
    for k in splits:
        out.append((a0, k))
        a0 += k
    return out


def run_batch_host(lib, api, params, kind, n, nctx, fpc, cap, srcs, ts_start=5000, primary_g=None, splits=None):
    """primary_g: optional src -> g, set as the context's primary encoder
    parameter before each call (the CMP_GPU_AUTO_RICE rule).  splits: the
    acquisitions per cmp_gpu_compress call when the GPU side makes several
    calls on the same contexts (the loop order is then call by call, c-major
    inside a call); frames are returned in (context, acquisition) order."""
    sb = 4 if kind == "i16_in_i32" else 2
    pcs = _per_ctx(params, nctx)
    lib.set_timestamp_func(_ts_counter(ts_start))
    try:
        wbs = max(_work_size(lib, api, p, n * sb) for p in pcs)
        ctxs = [api.CmpContext() for _ in range(nctx)]
        wbs_bufs = [api.aligned_empty(max(wbs, 2), fill=0) for _ in range(nctx)]
        for c in range(nctx):
            w = _work_size(lib, api, pcs[c], n * sb)
            r = lib.initialise(ctxs[c], pcs[c], wbs_bufs[c] if w else None, w)
            assert not api.is_error(r), api.error_name(r)
        frames = [None] * (nctx * fpc)
        for a0, k in _calls(fpc, splits):
            for c in range(nctx):
                for a in range(a0, a0 + k):
                    dst = api.aligned_empty(cap + 64, fill=0xAB)
                    if primary_g is not None:
                        ctxs[c].params.primary_encoder_param = primary_g(srcs[c * fpc + a])
                    r = lib.compress(kind, ctxs[c], dst, cap, srcs[c * fpc + a])
                    frames[c * fpc + a] = (r, bytes(dst[:r]) if not api.is_error(r) else None)
        state = [(x.identifier, x.sequence_number, x.model_size, bytes(w[:wbs]))
                 for x, w in zip(ctxs, wbs_bufs)]
        return tuple(frames), tuple(state)
    finally:
        lib.set_timestamp_func(None)


def run_batch_gpu(lib, eng, api, params, kind, n, nctx, fpc, cap, srcs, ts_start=5000, flags=0, splits=None,
                  separate_work=False):
    """separate_work: each context's work buffer its own allocation, at
    uneven distances (the library then passes a pointer per context)."""
    import torch
    sb = 4 if kind == "i16_in_i32" else 2
    pcs = _per_ctx(params, nctx)
    nf = nctx * fpc
    stride = n * sb
    calls = _calls(fpc, splits)
    # batch order: call by call, c-major inside a call
    order = [c * fpc + a for a0, k in calls for c in range(nctx) for a in range(a0, a0 + k)]
    host_src = np.concatenate([np.ascontiguousarray(srcs[f]).view(np.uint8) for f in order])
    src = torch.from_numpy(host_src).cuda()
    dstride = (cap + 64 + 7) // 8 * 8
    dst = torch.full((nf * dstride,), 0xAB, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    lib.set_timestamp_func(_ts_counter(ts_start))
    try:
        wbs = max(_work_size(lib, api, p, stride) for p in pcs)
        wstride = (max(wbs, 2) + 15) // 16 * 16
        if separate_work:
            works = [torch.zeros(wstride + 4096 * (c % 3), dtype=torch.uint8, device="cuda") for c in range(nctx)]
            wptr = [t.data_ptr() for t in works]
        else:
            work = torch.zeros(nctx * wstride, dtype=torch.uint8, device="cuda")
            wptr = [work.data_ptr() + c * wstride for c in range(nctx)]
        ctxs = (api.CmpContext * nctx)()
        for c in range(nctx):
            w = _work_size(lib, api, pcs[c], stride)
            r = lib.initialise(ctxs[c], pcs[c], wptr[c] if w else None, w)
            assert not api.is_error(r), api.error_name(r)
        torch.cuda.synchronize()
        off = 0
        for a0, k in calls:
            r = eng.compress(ctxs, k, kind, src.data_ptr() + off * stride, stride, stride,
                             dst.data_ptr() + off * dstride, dstride, cap, sizes.data_ptr() + 4 * off, flags)
            assert r == 0, api.error_name(r)
            off += nctx * k
        assert eng.synchronize() == 0
        sz = sizes.cpu().numpy().astype(np.uint32)
        host = dst.cpu().numpy()
        wk = [t.cpu().numpy()[:wbs] for t in works] if separate_work else \
            [work.cpu().numpy()[c * wstride:c * wstride + wbs] for c in range(nctx)]
        frames = [None] * nf
        for j, f in enumerate(order):
            s = int(sz[j])
            frames[f] = (s, bytes(host[j * dstride:j * dstride + s]) if not api.is_error(s) else None)
        state = [(ctxs[c].identifier, ctxs[c].sequence_number, ctxs[c].model_size, bytes(wk[c]))
                 for c in range(nctx)]
        return tuple(frames), tuple(state)
    finally:
        lib.set_timestamp_func(None)
