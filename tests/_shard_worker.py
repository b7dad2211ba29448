"""Rank body for tests/test_shard_gloo.py (world-size-2 gloo on CPU).

Each rank encodes its shard of frames with the CPU oracle (test
infrastructure; on the GPU box the frames come from cmp_gpu_compress), then
the ranks run airs_compression_amd.shard.gather_frames_timed, and the root
checks every gathered frame against the oracle's encode of the whole set in
global frame order."""
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


def run(rank, world, port, nf, n, layout, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
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
        if mode == "patch_refused":
            try:
                shard.gather_frames_timed(dist, dst_t, stride, sizes_t, nf, rank, world, layout=layout,
                                          patch_base=0, params=api.CmpParams(**PARAMS, secondary_iterations=2))
            except ValueError as e:
                assert "identifier patching" in str(e)
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
