"""CMP_GPU_AUTO_RICE (the build-defined per-frame Rice k of BASELINE config 3)
against the oracle: k = orc_select_rice_k of the frame, then the oracle's
GOLOMB_ZERO encoder with g = 2^k.  Frames of up to AUTO_MAX_SPF segments
choose k inside the encode kernel (frame-major dispatch, 16 candidate granules
per segment); larger frames go through the sliced selection first.  Both paths,
both sample widths, NONE and DIFF, whole and partial segments, every k from 0
to 15 (the scale of the noise sweeps it), and frames holding the extreme
mapped value 65535 (v = 65536, the top histogram bin).  Bit-exact, with the
clock-derived identifier bytes 8-13 masked (one context: frame f is that
context's f-th primary pass)."""
import zlib

import numpy as np
import pytest

from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi
P = api.CmpParams
SEG16 = 4 * 4096  # samples per segment, 16-bit input (4 chunks)
SEG32 = 2 * 4096  # i16-in-i32 input (2 chunks)
AUTO_MAX_SPF = 32


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


def _frames(rng, kind, n, nf, extreme):
    """nf frames of a random walk / noise mix whose scale sweeps k = 0..15."""
    out = []
    for f in range(nf):
        scale = 2.0 ** rng.uniform(-1, 15.5)
        walk = rng.random() < 0.5
        x = rng.laplace(0, scale, n)
        if walk:
            x = np.cumsum(x) * 0.05
        x = np.clip(np.round(x), -32768, 32767).astype(np.int64)
        if extreme and f % 2 == 0:
            x[rng.integers(0, n, 3)] = -32768  # NONE: ZigZag 65535
            if n >= 2:
                i = int(rng.integers(1, n))
                x[i - 1], x[i] = 32767, -32768  # DIFF: residual -32768 (wraps) -> 65535 too
        if kind == "u16":
            out.append((x & 0xFFFF).astype(np.uint16))
        elif kind == "i16":
            out.append(x.astype(np.int16))
        else:  # i16 in i32: junk in the high half, which the encoder ignores
            hi = rng.integers(-30000, 30000, n).astype(np.int64) << 16
            out.append(((x & 0xFFFF) | hi).astype(np.int64).astype(np.int32))
    return out


def _oracle(orc, orc_ext, kind, pre, frames, checksum=0):
    want = []
    for x in frames:
        n = x.size
        k = orc_ext.orc_select_rice_k(np.ascontiguousarray(x).ctypes.data, n, 1 if kind == "i16_in_i32" else 0,
                                      pre, None)
        ctx = api.CmpContext()
        prm = P(primary_preprocessing=pre, primary_encoder_type=api.ENCODER_GOLOMB_ZERO,
                primary_encoder_param=1 << k, checksum_enabled=checksum)
        assert not api.is_error(orc.initialise(ctx, prm))
        cap = orc.compress_bound(2 * n)
        cap = cap if not api.is_error(cap) else 6 * n + 64  # past the 24-bit size field's worst case
        dst = api.aligned_empty(cap)
        r = orc.compress(kind, ctx, dst, cap, x)
        assert not api.is_error(r), api.error_name(r)
        want.append(bytes(dst[:r]))
    return want


def _gpu(prod, eng, kind, pre, frames, checksum=0):
    import torch
    n, nf = frames[0].size, len(frames)
    sb = 4 if kind == "i16_in_i32" else 2
    stride = (n * sb + 15) // 16 * 16  # 16-byte aligned frames (the FULL kernels when n fills segments)
    host = np.zeros(nf * stride, dtype=np.uint8)
    for f, x in enumerate(frames):
        host[f * stride:f * stride + n * sb] = np.ascontiguousarray(x).view(np.uint8)
    src = torch.from_numpy(host).cuda()
    cap = prod.compress_bound(2 * n)
    cap = cap if not api.is_error(cap) else 6 * n + 64
    dstride = (cap + 7) // 8 * 8
    dst = torch.full((nf * dstride,), 0xAB, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = (api.CmpContext * 1)()
    # the configured g is ignored by AUTO_RICE (any valid g)
    prm = P(primary_preprocessing=pre, primary_encoder_type=api.ENCODER_GOLOMB_ZERO, primary_encoder_param=7,
            checksum_enabled=checksum)
    assert not api.is_error(prod.initialise(ctxs[0], prm))
    torch.cuda.synchronize()
    r = eng.compress(ctxs, nf, kind, src.data_ptr(), stride, n * sb, dst.data_ptr(), dstride, cap,
                     sizes.data_ptr(), 1)
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
for kind, seg in (("u16", SEG16), ("i16", SEG16), ("i16_in_i32", SEG32)):
    for pre in (0, 1):
        for n in (1, 7, 4096, seg - 1, seg, 3 * seg + 517, 4 * seg, AUTO_MAX_SPF * seg,
                  AUTO_MAX_SPF * seg + 100):
            CASES.append((kind, pre, n))
# cfg2-shaped frames (4 Mi samples, 256 segments) and 1 Mi i16-in-i32 samples:
# the sliced selection (one workgroup per 32 Ki-sample slice, not per frame)
CASES += [("u16", 1, 4 << 20), ("i16", 0, 4 << 20), ("i16_in_i32", 1, 1 << 20)]


@pytest.mark.parametrize("kind,pre,n", CASES)
def test_autorice_vs_oracle(prod, eng, orc, orc_ext, kind, pre, n):
    rng = np.random.default_rng(zlib.crc32(f"{kind}/{pre}/{n}".encode()))
    budget = 3 << 20  # samples per case (oracle time)
    nf = int(max(2, min(24, budget // max(n, 1))))
    frames = _frames(rng, kind, n, nf, extreme=True)
    want = _oracle(orc, orc_ext, kind, pre, frames)
    got = _gpu(prod, eng, kind, pre, frames)
    bad = [f for f in range(nf) if _mask(got[f]) != _mask(want[f])]
    assert not bad, (f"frames {bad[:8]} differ; g gpu/oracle "
                     f"{[(api.parse_header(got[f])['encoder_param'], api.parse_header(want[f])['encoder_param']) for f in bad[:4]]}")


@pytest.fixture(scope="module")
def eng_x(prod):
    """an engine marked CMP_GPU_OPT_EXCLUSIVE: frames of 9 .. AUTO_MAX_SPF
    segments choose k inside the encode kernel (without the option they take
    the selection kernel first)"""
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    assert e.set_option(load_pkg().OPT_EXCLUSIVE, 1) == 0
    yield e
    e.close()


@pytest.mark.parametrize("kind,pre,n", [("u16", 1, 9 * SEG16), ("i16", 0, 17 * SEG16 + 3), ("u16", 0, AUTO_MAX_SPF * SEG16),
                                        ("i16_in_i32", 1, AUTO_MAX_SPF * SEG32), ("u16", 1, AUTO_MAX_SPF * SEG16 + 1)])
def test_autorice_exclusive_engine_vs_oracle(prod, eng_x, orc, orc_ext, kind, pre, n):
    rng = np.random.default_rng(zlib.crc32(f"x/{kind}/{pre}/{n}".encode()))
    frames = _frames(rng, kind, n, 6, extreme=True)
    want = _oracle(orc, orc_ext, kind, pre, frames)
    got = _gpu(prod, eng_x, kind, pre, frames)
    bad = [f for f in range(len(frames)) if _mask(got[f]) != _mask(want[f])]
    assert not bad, f"frames {bad[:8]} differ"


def test_autorice_beside_other_kernels(prod, eng, orc, orc_ext):
    """a cfg3-shaped AUTO batch (frames of 64 Ki u16, 4
    segments, DIFF; the fused selection, whose segments meet at their frame's
    candidate barrier) on an engine NOT marked exclusive, while kernels on a
    second stream keep the CUs busy: bit-exact, and no look-back or barrier
    give-up (CMP_ERR_INT_BITSTREAM from cmp_gpu_synchronize, which _gpu
    checks)."""
    import threading

    import torch
    rng = np.random.default_rng(7)
    frames = _frames(rng, "u16", 4 * SEG16, 96, extreme=False)
    want = _oracle(orc, orc_ext, "u16", 1, frames)
    side = torch.cuda.Stream()
    buf = torch.empty(1 << 27, dtype=torch.float32, device="cuda")  # 512 MiB of elementwise work per op
    stop = threading.Event()

    def load():
        with torch.cuda.stream(side):
            while not stop.is_set():
                buf.mul_(1.0001).add_(0.5)
                side.synchronize()
    t = threading.Thread(target=load)
    t.start()
    try:
        got = [_gpu(prod, eng, "u16", 1, frames) for _ in range(3)]
    finally:
        stop.set()
        t.join()
    for g in got:
        bad = [f for f in range(len(frames)) if _mask(g[f]) != _mask(want[f])]
        assert not bad, f"frames {bad[:8]} differ"


def test_autorice_k_range(prod, eng, orc, orc_ext):
    """The sweep reaches every k: scales 2^-1 .. 2^15.5 over 64 frames."""
    rng = np.random.default_rng(11)
    frames = _frames(rng, "u16", SEG16, 64, extreme=False)
    got = _gpu(prod, eng, "u16", 0, frames)
    want = _oracle(orc, orc_ext, "u16", 0, frames)
    assert [_mask(g) for g in got] == [_mask(w) for w in want]
    ks = {api.parse_header(g)["encoder_param"].bit_length() - 1 for g in got}
    assert len(ks) >= 12, sorted(ks)


AUTO_BATCH = [  # (kind, n, fallback, flags beyond AUTO_RICE)
    ("u16", AUTO_MAX_SPF * SEG16 + 100, 1, 0),  # device exact mode, sliced selection per launch
    ("u16", AUTO_MAX_SPF * SEG16 + 100, 1, 0x2),  # the same, host-stepped
    ("i16_in_i32", 3 * SEG32 + 5, 1, 0),  # device exact mode, k chosen in the encode kernel
    ("i16", 2 * SEG16, 0, 0),  # asynchronous mode (one launch per acquisition step: no walk)
]


@pytest.mark.parametrize("kind,n,fallback,extra", AUTO_BATCH)
def test_autorice_model_batch(prod, eng, orc, orc_ext, kind, n, fallback, extra):
    """AUTO_RICE in multi-context batches with a MODEL secondary pass: the
    primary (DIFF) passes take the per-frame g of the rule, the MODEL passes
    keep their configured g; contexts, models and fallbacks as the call loop
    with that g set before each call (identifiers included, unmasked).  Each
    launch selects g for its own frames only (the sliced selection over the
    launch's frame list)."""
    import batch_scenarios as bs
    rng = np.random.default_rng(n + extra)
    nctx, fpc = 2, 5
    frames = _frames(rng, kind, n, nctx * fpc, extreme=False)
    prm = P(primary_preprocessing=1, primary_encoder_type=api.ENCODER_GOLOMB_ZERO, primary_encoder_param=4,
            secondary_iterations=2, secondary_preprocessing=3, secondary_encoder_type=api.ENCODER_GOLOMB_ZERO,
            secondary_encoder_param=8, model_rate=9, checksum_enabled=1, uncompressed_fallback_enabled=fallback)
    cap = 26 + 6 * n

    def primary_g(x):
        return 1 << orc_ext.orc_select_rice_k(np.ascontiguousarray(x).ctypes.data, n,
                                              1 if kind == "i16_in_i32" else 0, 1, None)
    want = bs.run_batch_host(orc, api, prm, kind, n, nctx, fpc, cap, frames, primary_g=primary_g)
    got = bs.run_batch_gpu(prod, eng, api, prm, kind, n, nctx, fpc, cap, frames, flags=1 | extra)
    assert got[1] == want[1]
    bad = [f for f in range(nctx * fpc) if got[0][f] != want[0][f]]
    assert not bad, f"frames {bad} differ"


# IWT passes (round 5): k from the pass's residuals, the IWT coefficients.
# The oracle side runs the IWT pass once to get them (its work buffer holds
# the coefficients afterwards, preprocess.c:321-353), picks k with
# orc_select_rice_k over them as 16-bit NONE residuals, then encodes with 2^k.
IWT_CASES = [("u16", 65536, 0), ("u16", 1 << 20, 0), ("i16", 5000, 0), ("i16_in_i32", 70000, 0),
             ("u16", 65536, 1), ("i16", 4160, 1)]


@pytest.mark.parametrize("kind,n,fallback", IWT_CASES)
def test_autorice_iwt_vs_oracle(prod, eng, orc, orc_ext, kind, n, fallback):
    import torch
    rng = np.random.default_rng(zlib.crc32(f"iwt/{kind}/{n}/{fallback}".encode()))
    nf = int(max(2, min(12, (2 << 20) // n)))
    frames = _frames(rng, kind, n, nf, extreme=True)
    if fallback:  # a few noise frames that fall back
        for f in range(0, nf, 3):
            x = rng.integers(-32768, 32768, n)
            frames[f] = (x & 0xFFFF).astype(np.uint16) if kind == "u16" else x.astype(
                np.int16 if kind == "i16" else np.int32)
    sb = 4 if kind == "i16_in_i32" else 2
    wbs = (2 * n + 15) // 16 * 16
    raw = 16 + 2 * n
    want = []
    for x in frames:
        c0, wb = api.CmpContext(), api.aligned_empty(wbs)
        prm = P(primary_preprocessing=api.PREPROCESS_IWT, primary_encoder_type=api.ENCODER_GOLOMB_ZERO,
                primary_encoder_param=1)
        assert not api.is_error(orc.initialise(c0, prm, wb, wbs))
        cap = 6 * n + 64
        d = api.aligned_empty(cap)
        assert not api.is_error(orc.compress(kind, c0, d, cap, x))
        k = orc_ext.orc_select_rice_k(wb.ctypes.data, n, 0, api.PREPROCESS_NONE, None)
        c1, wb1 = api.CmpContext(), api.aligned_empty(wbs)
        prm = P(primary_preprocessing=api.PREPROCESS_IWT, primary_encoder_type=api.ENCODER_GOLOMB_ZERO,
                primary_encoder_param=1 << k, uncompressed_fallback_enabled=fallback)
        assert not api.is_error(orc.initialise(c1, prm, wb1, wbs))
        ocap = raw if fallback else cap
        r = orc.compress(kind, c1, d, ocap, x)
        assert not api.is_error(r), api.error_name(r)
        want.append(bytes(d[:r]))
    # the GPU: one context, nf acquisitions, AUTO_RICE (the configured g is ignored)
    stride = (n * sb + 15) // 16 * 16
    host = np.zeros(nf * stride, dtype=np.uint8)
    for f, x in enumerate(frames):
        host[f * stride:f * stride + n * sb] = np.ascontiguousarray(x).view(np.uint8)
    src = torch.from_numpy(host).cuda()
    cap = raw if fallback else 6 * n + 64
    dstride = (6 * n + 64 + 7) // 8 * 8
    dst = torch.full((nf * dstride,), 0xAB, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    work = torch.zeros(wbs, dtype=torch.uint8, device="cuda")
    ctxs = (api.CmpContext * 1)()
    prm = P(primary_preprocessing=api.PREPROCESS_IWT, primary_encoder_type=api.ENCODER_GOLOMB_ZERO,
            primary_encoder_param=7, uncompressed_fallback_enabled=fallback)
    assert not api.is_error(prod.initialise(ctxs[0], prm, work.data_ptr(), wbs))
    torch.cuda.synchronize()
    r = eng.compress(ctxs, nf, kind, src.data_ptr(), stride, n * sb, dst.data_ptr(), dstride, cap,
                     sizes.data_ptr(), 1)
    assert r == 0, api.error_name(r)
    assert eng.synchronize() == 0
    sz = sizes.cpu().numpy().astype(np.uint32)
    out = dst.cpu().numpy()
    got = [bytes(out[f * dstride:f * dstride + int(sz[f])]) for f in range(nf)]
    bad = [f for f in range(nf) if _mask(got[f]) != _mask(want[f])]
    assert not bad, (f"frames {bad[:8]} differ; g gpu/oracle "
                     f"{[(api.parse_header(got[f])['encoder_param'], api.parse_header(want[f])['encoder_param']) for f in bad[:4] if len(got[f]) >= 22]}")
    if fallback:
        assert any(api.parse_header(w)["encoder_type"] == api.ENCODER_UNCOMPRESSED for w in want)
