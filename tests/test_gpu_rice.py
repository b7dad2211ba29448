"""The Rice/ZERO frame kernel (enc_rice.hip) against the
oracle: 16-bit frames of whole 16 Ki-sample segments, NONE and DIFF,
GOLOMB_ZERO with g = 2^k for k = 0 .. 7 (the kernel's range) and 8 (past it:
encode_kernel), with and without checksums.

The data are chosen for the kernel's special steps:
  * laplace noise at the scale of g (the common case: every pair fits 32 bits
    but the escapes);
  * smooth data with single-sample outliers: each outlier gives two adjacent
    zero escapes, a pair of 2 (k + 17) bits, re-coded from the table;
  * uniform random samples: escapes everywhere, more bits than the arena
    holds, so the segment is stored chunk by chunk after its look-back;
  * constant frames (every sample the shortest code) and the extreme mapped
    value 65535.
Frames of 40 segments put the scalar first look-back round (16 granules)
and the vector rounds behind it to work.  Bit-exact, with the clock-derived
identifier bytes 8-13 masked (one context: frame f is its f-th primary pass).
Reference: lib/compress/cmp.c:296-312, encoder.c:327-351,
bitstream_writer.h:124-158."""
import zlib

import numpy as np
import pytest

from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi
P = api.CmpParams
SEG = 16384


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


def _frame(rng, kind, n, k, data):
    if data == "laplace":
        x = np.round(rng.laplace(0, 2.0 ** k, n)).astype(np.int64)
        x = np.cumsum(x) if rng.random() < 0.5 else x
    elif data == "outliers":
        x = np.round(rng.laplace(0, 2.0 ** k, n)).astype(np.int64) + 16384
        idx = rng.integers(0, n, max(1, n // 700))
        x[idx] = rng.integers(0, 65536, idx.size)
        x[::4099] = 0x8000 + x[::4099]  # an outlier at every alignment
    elif data == "uniform":
        x = rng.integers(0, 65536, n)
    elif data == "const":
        x = np.full(n, int(rng.integers(0, 65536)), dtype=np.int64)
    else:  # extreme: the largest mapped value, NONE and DIFF
        x = np.where(np.arange(n) % 2 == 0, 32767, -32768).astype(np.int64)
        x[rng.integers(0, n, 50)] = 0
    x = x & 0xFFFF
    return x.astype(np.uint16) if kind == "u16" else x.astype(np.uint16).view(np.int16)


def _oracle(orc, kind, pre, g, frames, checksum):
    want = []
    for x in frames:
        ctx = api.CmpContext()
        prm = P(primary_preprocessing=pre, primary_encoder_type=api.ENCODER_GOLOMB_ZERO, primary_encoder_param=g,
                checksum_enabled=checksum)
        assert not api.is_error(orc.initialise(ctx, prm))
        cap = orc.compress_bound(2 * x.size)
        dst = api.aligned_empty(cap)
        r = orc.compress(kind, ctx, dst, cap, x)
        assert not api.is_error(r), api.error_name(r)
        want.append(bytes(dst[:r]))
    return want


def _gpu(prod, eng, kind, pre, g, frames, checksum):
    import torch
    n, nf = frames[0].size, len(frames)
    stride = 2 * n
    host = np.zeros(nf * stride, dtype=np.uint8)
    for f, x in enumerate(frames):
        host[f * stride:(f + 1) * stride] = np.ascontiguousarray(x).view(np.uint8)
    src = torch.from_numpy(host).cuda()
    cap = prod.compress_bound(2 * n)
    dstride = (cap + 7) // 8 * 8
    dst = torch.full((nf * dstride,), 0xAB, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = (api.CmpContext * 1)()
    prm = P(primary_preprocessing=pre, primary_encoder_type=api.ENCODER_GOLOMB_ZERO, primary_encoder_param=g,
            checksum_enabled=checksum)
    assert not api.is_error(prod.initialise(ctxs[0], prm))
    torch.cuda.synchronize()
    r = eng.compress(ctxs, nf, kind, src.data_ptr(), stride, 2 * n, dst.data_ptr(), dstride, cap, sizes.data_ptr(), 0)
    assert r == 0, api.error_name(r)
    assert eng.synchronize() == 0
    sz = sizes.cpu().numpy().astype(np.uint32)
    out = dst.cpu().numpy()
    got = []
    for f in range(nf):
        assert not api.is_error(int(sz[f])), api.error_name(int(sz[f]))
        got.append(bytes(out[f * dstride:f * dstride + int(sz[f])]))
    return got


def _mask(b):
    b = bytearray(b)
    b[8:14] = b"\0" * 6
    return bytes(b)


CASES = []
for k in range(0, 9):
    for pre in (0, 1):
        for data in ("laplace", "outliers", "uniform", "const", "extreme"):
            CASES.append((k, pre, data))


@pytest.mark.parametrize("k,pre,data", CASES)
def test_rice_kernel_vs_oracle(prod, eng, orc, k, pre, data):
    rng = np.random.default_rng(zlib.crc32(f"{k}/{pre}/{data}".encode()))
    kind = "u16" if (k + pre) % 2 == 0 else "i16"
    checksum = (k + len(data)) % 3 == 0
    # segments per frame: 1, 3 and 40 (the scalar look-back round), ragged batch
    shapes = [(1, 5), (3, 3), (40, 2)] if data in ("laplace", "outliers") else [(1, 3), (3, 2)]
    for spf, nf in shapes:
        n = spf * SEG
        frames = [_frame(rng, kind, n, k, data) for _ in range(nf)]
        want = _oracle(orc, kind, pre, 1 << k, frames, checksum)
        got = _gpu(prod, eng, kind, pre, 1 << k, frames, checksum)
        bad = [f for f in range(nf) if _mask(got[f]) != _mask(want[f])]
        assert not bad, (spf, bad, [(len(got[f]), len(want[f])) for f in bad])


def test_rice_kernel_host_api(prod, orc):
    """The host API (cmp_compress_u16 stages the frame to the device) on frames
    of whole segments, one context across calls: same frames and sequence."""
    rng = np.random.default_rng(5)
    for pre, g in ((1, 32), (0, 8), (1, 1)):
        outs = []
        for lib in (prod, orc):
            lib.set_timestamp_func(lambda: (3, 4))
            ctx = api.CmpContext()
            assert not api.is_error(lib.initialise(ctx, P(primary_preprocessing=pre, primary_encoder_type=1,
                                                          primary_encoder_param=g, checksum_enabled=1)))
            res = []
            for i in range(3):
                x = _frame(np.random.default_rng(100 + i), "u16", 2 * SEG, 5, "outliers")
                cap = lib.compress_bound(x.nbytes)
                dst = api.aligned_empty(cap)
                r = lib.compress_u16(ctx, dst, cap, x)
                res.append((r, bytes(dst[:r]) if not api.is_error(r) else None))
            lib.set_timestamp_func(None)
            outs.append(res)
        assert outs[0] == outs[1], (pre, g)
    _ = rng


def test_rice_kernel_small_capacity(prod, eng, orc):
    """A capacity below the compressed size: the hardware range check drops
    the words past it and the frame reports CMP_ERR_DST_TOO_SMALL, as the
    encode kernel does."""
    import torch
    n = 2 * SEG
    x = _frame(np.random.default_rng(9), "u16", n, 5, "laplace")
    ctxs = (api.CmpContext * 1)()
    prm = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32)
    assert not api.is_error(prod.initialise(ctxs[0], prm))
    src = torch.from_numpy(x.view(np.uint8).copy()).cuda()
    for cap in (64, 4096, 20000):
        dst = torch.zeros(cap + 64, dtype=torch.uint8, device="cuda")
        sizes = torch.zeros(1, dtype=torch.int32, device="cuda")
        r = eng.compress(ctxs, 1, "u16", src.data_ptr(), 2 * n, 2 * n, dst.data_ptr(), cap + 64, cap,
                         sizes.data_ptr(), 0)
        assert r == 0
        assert eng.synchronize() == 0
        s = int(sizes.cpu().numpy().astype(np.uint32)[0])
        assert api.is_error(s) and api.error_name(s) == "DST_TOO_SMALL", api.error_name(s)
        assert not dst[cap:].any().item()  # nothing past the capacity
