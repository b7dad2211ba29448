"""GPU decoder (cmp_gpu_decompress).  The reference has
no decoder, so parity is anchored on the encoder: frames written by the CPU
oracle's encoder must decode to the samples it encoded (and to what the
oracle's own decoder, orc_decode, returns), and frames written by the GPU
encoder must round-trip at BASELINE sizes.  Bit-exact (16-bit samples)."""
import numpy as np
import pytest

import configs
import scenarios
from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi


@pytest.fixture(scope="module")
def gpu(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    return prod


@pytest.fixture(scope="module")
def eng(gpu):
    e = gpu.engine()
    yield e
    e.close()


def gpu_decode(eng, frames, n_max, cap=None):
    """Upload frames (bytes) at a common stride, decode on the GPU; returns
    (status list, samples per frame as uint16 arrays)."""
    import torch
    cap = cap or max(22, max(len(f) for f in frames))
    cap = (cap + 7) // 8 * 8
    nf = len(frames)
    host = np.zeros(nf * cap, dtype=np.uint8)
    for i, f in enumerate(frames):
        host[i * cap:i * cap + len(f)] = np.frombuffer(f, dtype=np.uint8)
    src = torch.from_numpy(host).cuda()
    dstride = 2 * max(n_max, 1)
    dst = torch.zeros(nf * dstride // 2, dtype=torch.int16, device="cuda")
    st = torch.zeros(nf, dtype=torch.int32, device="cuda")
    assert eng.decompress(src.data_ptr(), cap, cap, nf, dst.data_ptr(), dstride, n_max, st.data_ptr()) == 0
    assert eng.synchronize() == 0
    status = [int(s) & 0xFFFFFFFF for s in st.cpu().numpy()]
    out = dst.cpu().numpy().view(np.uint16)
    return status, [out[i * (dstride // 2):(i + 1) * (dstride // 2)] for i in range(nf)]


def oracle_frame(orc, params, kind, x):
    ctx = api.CmpContext()
    assert not api.is_error(orc.initialise(ctx, params))
    cap = 26 + 6 * len(x) + 64
    dst = api.aligned_empty(cap)
    r = orc.compress(kind, ctx, dst, cap, x)
    assert not api.is_error(r), api.error_name(r)
    return bytes(dst[:r])


def test_decode_vs_oracle_frames(eng, orc, orc_ext):
    """Random NONE / DIFF frames of every encoder, Golomb parameters from 1 to
    65535 (Rice and general), outliers, checksums, sizes from 1 to 70 k."""
    import random
    rng = random.Random(11)
    frames, want = [], []
    for trial in range(160):
        kind = rng.choice(scenarios.KINDS)
        n = rng.choice([1, 2, 3, 7, 100, 333, 2048, 4097, 9000, 70001])
        enc = rng.choice([0, 1, 2])
        p = api.CmpParams(primary_preprocessing=rng.choice([0, 1]), primary_encoder_type=enc,
                          primary_encoder_param=rng.choice([1, 2, 3, 7, 8, 10, 32, 100, 1055, 4096, 65535]),
                          primary_encoder_outlier=rng.choice([1, 5, 107, 1000, 2**32 - 1]),
                          checksum_enabled=rng.choice([0, 1]))
        x = scenarios.make_src(kind, n, rng, rng.choice([1, 50, 3000, 30000]))
        fr = oracle_frame(orc, p, kind, x)
        out = np.zeros(n, dtype=np.uint16)
        assert orc_ext.orc_decode(np.frombuffer(fr, dtype=np.uint8).ctypes.data, len(fr), None,
                                  out.ctypes.data, n) == n
        assert np.array_equal(out, (np.asarray(x).astype(np.int64) & 0xFFFF).astype(np.uint16))
        frames.append(fr)
        want.append(out)
    status, outs = gpu_decode(eng, frames, 70001)
    for i, (s, w) in enumerate(zip(status, want)):
        assert s == len(w), (i, api.error_name(s) if api.is_error(s) else s)
        assert np.array_equal(outs[i][:len(w)], w), i


@pytest.mark.parametrize("name", ["cfg2_64Mi", "cfg4_8192"])
def test_decode_roundtrip_gpu_frames(gpu, eng, orc_ext, name):
    """Size-independent property at BASELINE size: decode(encode(x)) == x for
    every frame the GPU encoder wrote (cfg4: the first 1024 frames)."""
    import torch
    cfg = dict(configs.CONFIGS[name])
    if name == "cfg4_8192":
        cfg["nctx"], cfg["fpc"] = 1, 1024
    frames, _, _ = configs.gpu_frames(gpu, eng, cfg)
    n = cfg["n"]
    status, outs = gpu_decode(eng, frames, n)
    assert status == [n] * len(frames)
    src = torch.empty(len(frames) * 2 * n, dtype=torch.uint8, device="cuda")
    assert eng.synthesize(src.data_ptr(), 2, cfg["seed"], 0, n, len(frames), 2 * n, cfg["W"]) == 0
    x = src.cpu().numpy().view(np.uint16).reshape(len(frames), n)
    for i in range(len(frames)):
        assert np.array_equal(outs[i][:n], x[i]), i


def test_decode_rejects(eng, orc):
    """Frames the decoder does not take or cannot parse: MODEL / IWT
    preprocessing, a broken header, a truncated payload."""
    rng = np.random.default_rng(3)
    x = (np.cumsum(rng.integers(-50, 50, 5000)) & 0xFFFF).astype(np.uint16)
    good = oracle_frame(orc, api.CmpParams(primary_preprocessing=1, primary_encoder_type=1,
                                           primary_encoder_param=16), "u16", x)
    bad_hdr = bytearray(good)
    bad_hdr[1] ^= 0x55  # version id
    trunc = bytearray(good[:200])  # keep the header's sizes, cut the payload
    trunc[2:5] = (200).to_bytes(3, "big")
    model = bytearray(good)
    model[15] = (3 << 4) | (model[15] & 0x0F)  # MODEL preprocessing: needs the model, not decoded
    unknown = [bytearray(good) for _ in range(12)]  # preprocessing 4..15: no such method
    for p, u in zip(range(4, 16), unknown):
        u[15] = (p << 4) | (u[15] & 0x0F)
    frames = [good, bytes(bad_hdr), bytes(trunc), bytes(model)] + [bytes(u) for u in unknown]
    status, outs = gpu_decode(eng, frames, 5000, cap=len(good) + 8)
    assert status[0] == 5000 and np.array_equal(outs[0][:5000], x)
    assert api.error_name(status[1]) == "INT_HDR"
    assert api.error_name(status[2]) == "INT_BITSTREAM"
    assert api.error_name(status[3]) == "PARAMS_INVALID"
    assert [api.error_name(s) for s in status[4:]] == ["INT_HDR"] * 12


def test_decode_model_frames(eng, orc):
    """MODEL frames decode against the model each was encoded with: the work
    buffer as the oracle held it before the call (preprocess.c:406-411)."""
    import torch
    rng = np.random.default_rng(5)
    frames, models, xs = [], [], []
    for trial in range(6):
        n = int(rng.choice([1, 17, 4096, 9001]))
        p = api.CmpParams(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
                          secondary_iterations=3, secondary_preprocessing=3,
                          secondary_encoder_type=int(rng.choice([0, 1, 2])), secondary_encoder_param=8,
                          secondary_encoder_outlier=107, model_rate=int(rng.choice([0, 11, 16])))
        ctx = api.CmpContext()
        wbs = orc.cal_work_buf_size(p, 2 * n)
        wb = api.aligned_empty(wbs, fill=0)
        assert not api.is_error(orc.initialise(ctx, p, wb, wbs))
        base = np.cumsum(rng.integers(-300, 300, n))
        for step in range(4):
            x = ((base + rng.integers(-40, 40, n)) & 0xFFFF).astype(np.uint16)
            before = np.frombuffer(bytes(wb[:2 * n]), dtype=np.uint16).copy()
            cap = 26 + 6 * n + 64
            dst = api.aligned_empty(cap)
            r = orc.compress_u16(ctx, dst, cap, x)
            assert not api.is_error(r), api.error_name(r)
            if step:  # secondary (MODEL) passes
                frames.append(bytes(dst[:r]))
                models.append(before)
                xs.append(x)
    nmax = max(len(x) for x in xs)
    mod = np.zeros((len(frames), nmax), dtype=np.uint16)
    for i, m in enumerate(models):
        mod[i, :len(m)] = m
    dmod = torch.from_numpy(mod.view(np.int16)).cuda()
    import types
    eng2 = types.SimpleNamespace(decompress=lambda *a: eng.decompress(*a, dmod.data_ptr(), 2 * nmax),
                                 synchronize=eng.synchronize)
    status, outs = gpu_decode(eng2, frames, nmax)
    for i, x in enumerate(xs):
        assert status[i] == len(x), (i, api.error_name(status[i]) if api.is_error(status[i]) else status[i])
        assert np.array_equal(outs[i][:len(x)], x), i


def test_decode_iwt_frames(eng, orc):
    """IWT frames: the inverse transform (levels from the largest stride down)
    restores the samples exactly; whole-frame LDS kernel up to 64 Ki samples,
    per-level launches above."""
    rng = np.random.default_rng(9)
    frames, xs = [], []
    for n in (1, 2, 3, 5, 7, 8, 100, 4097, 65536, 65537, 200001):
        for enc, g in ((1, 16), (2, 10), (0, 1)):
            p = api.CmpParams(primary_preprocessing=2, primary_encoder_type=enc, primary_encoder_param=g,
                              primary_encoder_outlier=200)
            ctx = api.CmpContext()
            wbs = orc.cal_work_buf_size(p, 2 * n)
            wb = api.aligned_empty(wbs, fill=0)
            assert not api.is_error(orc.initialise(ctx, p, wb, wbs))
            x = ((np.cumsum(rng.integers(-500, 500, n)) + rng.integers(-30000, 30000)) & 0xFFFF).astype(np.uint16)
            cap = 26 + 6 * n + 64
            dst = api.aligned_empty(cap)
            r = orc.compress_u16(ctx, dst, cap, x)
            assert not api.is_error(r), api.error_name(r)
            frames.append(bytes(dst[:r]))
            xs.append(x)
    status, outs = gpu_decode(eng, frames, max(len(x) for x in xs))
    for i, x in enumerate(xs):
        assert status[i] == len(x), (i, api.error_name(status[i]) if api.is_error(status[i]) else status[i])
        assert np.array_equal(outs[i][:len(x)], x), (i, len(x))
