"""Rank body for tests/test_shard_gloo.py (world-size-2 gloo on CPU).

Each rank encodes its shard of frames with the CPU oracle (test
infrastructure; on the GPU box the frames come from cmp_gpu_compress), then
the ranks run airs_compression_amd.shard.gather_frames_timed, and the root
checks every gathered frame against the oracle's encode of the whole set in
global frame order.

Modes "fallback" and "streams" pass each frame's identifier-draw count (what
cmp_gpu_batch.draws reports; counted here from the timestamp callback) and
compare the patched identifiers UNMASKED with one process's call loop:
  fallback  frames round robin, primary passes with the uncompressed fallback
            (noise frames fall back: three draws), against ONE context over
            all frames in global order;
  streams   streams of FPC frames, stream s on rank s mod 2, MODEL secondary
            passes and the fallback, against one context per stream, the
            contexts initialised in stream order and compressed stream-major
            (cmp_gpu_compress's call order)."""
import os

import numpy as np
import torch
import torch.distributed as dist

import conftest

PARAMS = dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32)


def encode(orc, orc_ext, api, frames, n, seed):
    cap = orc.compress_bound(2 * n)
    stride = (cap + 7) // 8 * 8
    dst = np.zeros(stride * max(len(frames), 1), dtype=np.uint8)
    sizes = np.zeros(len(frames), dtype=np.int32)
    ctx = api.CmpContext()
    assert not api.is_error(orc.initialise(ctx, api.CmpParams(**PARAMS)))
    x = np.empty(n, dtype=np.uint16)
    for j, f in enumerate(frames):
        orc_ext.orc_synth_u16(seed, f, n, 32, x.ctypes.data)
        buf = api.aligned_empty(cap)
        r = orc.compress_u16(ctx, buf, cap, x)
        assert not api.is_error(r), api.error_name(r)
        dst[j * stride:j * stride + r] = buf[:r]
        sizes[j] = r
    return dst, stride, sizes


class Counter:
    """timestamp callback 1000+1, 1000+2, ... counting its calls"""

    def __init__(self):
        self.v = 1000
        self.calls = 0

    def __call__(self):
        self.v += 1
        self.calls += 1
        return (self.v >> 16, self.v & 0xFFFF)


FB_PARAMS = dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=4,
                 uncompressed_fallback_enabled=1, checksum_enabled=1)
ST_PARAMS = dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=3,
                 secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
                 secondary_encoder_outlier=107, model_rate=11, uncompressed_fallback_enabled=1)
FPC = 5


def synth(g, n):
    """frame g: a random walk, every third frame noise (it falls back)"""
    rng = np.random.default_rng(1000 + g)
    if g % 3 == 2:
        return rng.integers(0, 65536, n).astype(np.uint16)
    return (np.cumsum(rng.integers(-3, 4, n)) & 0xFFFF).astype(np.uint16)


def encode_units(orc, api, params, units, n):
    """units: lists of global frame numbers, one context each (in order);
    returns dst, stride, sizes, draws (in the units' frame order) and the
    context count drawn at initialisation"""
    cap = orc.compress_bound(2 * n)
    stride = (cap + 7) // 8 * 8
    frames = [g for u in units for g in u]
    dst = np.zeros(stride * max(len(frames), 1), dtype=np.uint8)
    sizes = np.zeros(len(frames), dtype=np.int32)
    draws = np.zeros(len(frames), dtype=np.uint8)
    cnt = Counter()
    orc.set_timestamp_func(cnt)
    try:
        prm = api.CmpParams(**params)
        ctxs, works = [], []
        for _ in units:
            ctx = api.CmpContext()
            wbs = orc.cal_work_buf_size(prm, 2 * n)
            wb = api.aligned_empty(max(wbs, 2), fill=0) if wbs else None
            assert not api.is_error(orc.initialise(ctx, prm, wb, wbs))
            ctxs.append(ctx)
            works.append(wb)
        j = 0
        for ctx, u in zip(ctxs, units):
            for g in u:
                x = synth(g, n)
                buf = api.aligned_empty(cap)
                before = cnt.calls
                r = orc.compress_u16(ctx, buf, cap, x)
                assert not api.is_error(r), api.error_name(r)
                draws[j] = cnt.calls - before
                dst[j * stride:j * stride + r] = buf[:r]
                sizes[j] = r
                j += 1
    finally:
        orc.set_timestamp_func(None)
    return dst, stride, sizes, draws


def run_draws(rank, world, nf, n, mode):
    pkg = conftest.load_pkg()
    api = pkg.cmpapi
    shard = pkg.shard
    orc = api.CmpLib(conftest.ORC_PATH)
    if mode == "fallback":
        layout, fpc, params = "roundrobin", 1, FB_PARAMS
        mine = shard.rank_frames(nf * world, rank, world, layout)
        units = [mine]  # one context per rank, its frames in local order
    else:
        layout, fpc, params = "streams", FPC, ST_PARAMS
        mine = shard.rank_frames(nf * world, rank, world, layout, fpc)
        units = [mine[i:i + fpc] for i in range(0, len(mine), fpc)]
    dst, stride, sizes, draws = encode_units(orc, api, params, units, n)
    if mode == "fallback" and rank == 0:
        assert (draws == 3).sum() >= 1  # fallbacks happened on this rank
    base = 1001 if mode == "fallback" else 1000 + (nf * world) // fpc
    stats, g = shard.gather_frames_timed(dist, torch.from_numpy(dst), stride, torch.from_numpy(sizes), len(mine),
                                         rank, world, layout=layout, patch_base=base, draws=torch.from_numpy(draws),
                                         fpc=fpc)
    if rank != 0:
        assert g is None
        return
    assert "draw counts" in stats["identifiers"]
    total = nf * world
    if mode == "fallback":
        want_units = [list(range(total))]
    else:
        want_units = [list(range(s * fpc, (s + 1) * fpc)) for s in range(total // fpc)]
    wdst, wstride, wsizes, wdraws = encode_units(orc, api, params, want_units, n)
    for f in range(total):
        got = bytes(g.frame(f).numpy().tobytes())
        want = bytes(wdst[f * wstride:f * wstride + int(wsizes[f])].tobytes())
        assert got == want, f"frame {f} differs from the one-process call loop (identifiers unmasked)"


def run(rank, world, port, nf, n, layout, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if mode in ("fallback", "streams"):
            run_draws(rank, world, nf, n, mode)
            return
        pkg = conftest.load_pkg()
        api = pkg.cmpapi
        shard = pkg.shard
        orc = api.CmpLib(conftest.ORC_PATH)
        import ctypes
        orc_ext = ctypes.CDLL(conftest.ORC_PATH, mode=ctypes.RTLD_LOCAL)
        orc_ext.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_void_p]
        seed = 0x5EED + n
        mine = shard.rank_frames(nf * world, rank, world, layout)
        dst, stride, sizes = encode(orc, orc_ext, api, mine, n, seed)
        dst_t = torch.from_numpy(dst)
        sizes_t = torch.from_numpy(sizes)
        if mode == "error":
            if rank == 1:
                sizes_t[nf - 1] = -7  # (uint32)-7: an error value in the size slot
            try:
                shard.gather_frames(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout)
            except RuntimeError as e:
                assert "error value" in str(e)
            else:
                raise AssertionError("error value was not reported")
            return
        if mode == "patch_refused_draws":
            # draw counts replace only the fallback restriction: a frame layout
            # with secondary passes is still refused (by the parameters, and by
            # a frame that made no draw), on every rank before any communication
            for prm, d in ((api.CmpParams(**PARAMS, secondary_iterations=2), torch.ones(nf, dtype=torch.uint8)),
                           (None, torch.tensor([1] + [0] * (nf - 1), dtype=torch.uint8))):
                try:
                    shard.gather_frames_timed(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout,
                                              patch_base=0, params=prm, draws=d)
                except ValueError as e:
                    assert "secondary" in str(e)
                else:
                    raise AssertionError("patching a frame layout with secondary passes was not refused")
            return
        if mode == "patch_refused_one_rank":
            # only rank 1's draws show a secondary pass (a 0): every rank must
            # raise, none may wait in the gather
            d = torch.ones(nf, dtype=torch.uint8)
            if rank == 1:
                d[nf // 2] = 0
            try:
                shard.gather_frames_timed(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout,
                                          patch_base=0, params=None, draws=d)
            except ValueError as e:
                assert ("secondary" in str(e)) or ("another rank" in str(e)), str(e)
            else:
                raise AssertionError(f"rank {rank}: a refusal on rank 1 alone did not stop this rank")
            return
        if mode == "patch_refused":
            try:
                shard.gather_frames_timed(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout,
                                          patch_base=0, params=api.CmpParams(**PARAMS, secondary_iterations=2))
            except ValueError as e:
                assert "draw counts" in str(e)
            else:
                raise AssertionError("patching frames with secondary passes was not refused")
            return
        stats, g = shard.gather_frames_timed(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout,
                                             patch_base=1000, params=api.CmpParams(**PARAMS))
        if rank != 0:
            assert g is None and stats is None
            return
        assert g.num_frames == nf * world
        assert stats["frames"] == nf * world and stats["bytes_total"] == int(g.data.numel())
        # the packing read only the compressed bytes (rounded up to 8 per frame)
        own = sizes_t[:nf].to(torch.int64)
        assert stats["root_pack_bytes_read"] == int(((own + 7) // 8 * 8).sum())
        assert stats["root_pack_bytes_read"] < int(own.sum()) + 8 * nf
        want_dst, wstride, want_sizes = encode(orc, orc_ext, api, list(range(nf * world)), n, seed)
        stream = g.ordered().numpy()
        pos = 0
        for f in range(nf * world):
            got = bytearray(g.frame(f).numpy().tobytes())
            want = bytearray(want_dst[f * wstride:f * wstride + int(want_sizes[f])].tobytes())
            assert int.from_bytes(got[8:14], "big") == 1000 + 1 + f, f
            got[8:14] = want[8:14] = b"\0" * 6
            assert got == want, f"frame {f} differs after the gather"
            assert bytes(stream[pos + 14:pos + len(got)]) == bytes(got[14:])
            pos += len(got)
        assert pos == stream.size
    finally:
        dist.destroy_process_group()
