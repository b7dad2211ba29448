"""GPU parity: the HIP path (libairscmp.so) against the oracle and the
reference's golden vectors.  Bit-exact everywhere (integer work)."""
import hashlib
import json
import os

import numpy as np
import pytest

import configs
import scenarios
from conftest import GOLDEN_DIR, ORC_PATH, load_pkg
from golden.gen_golden import run_kat

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi

with open(os.path.join(GOLDEN_DIR, "kats.json")) as f:
    KATS = json.load(f)["cases"]
with open(os.path.join(GOLDEN_DIR, "random_sequences.json")) as f:
    SEQS = json.load(f)["cases"]
with open(os.path.join(GOLDEN_DIR, "configs.json")) as f:
    CFG_GOLD = json.load(f)["configs"]


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


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_gpu(gpu, kat):
    assert run_kat(gpu, kat) == kat["expected"]


def test_random_sequences_gpu_vs_golden(gpu):
    """Reference digests for every golden scenario (IWT included): frames,
    context fields and the work buffer after every call."""
    bad, ran = [], 0
    for case in SEQS:
        params, kind, n = scenarios.random_case(api.CmpParams, case["trial"], allow_iwt=True)
        res = scenarios.run_sequence(gpu, params, kind, n, seed=case["trial"])
        ran += 1
        if hashlib.sha256(repr(res).encode()).hexdigest() != case["digest"]:
            bad.append(case["trial"])
    assert ran == len(SEQS) >= 400
    assert not bad, f"GPU differs from the reference on trials {bad[:10]}"


def test_random_sequences_gpu_vs_oracle(gpu, orc):
    bad = []
    for trial in range(20000, 20400):
        params, kind, n = scenarios.random_case(api.CmpParams, trial, allow_iwt=True)
        a = scenarios.run_sequence(gpu, params, kind, n, seed=trial)
        b = scenarios.run_sequence(orc, params, kind, n, seed=trial)
        if a != b:
            bad.append(trial)
    assert not bad, f"GPU differs from the oracle on trials {bad[:10]}"


def test_segment_boundaries_vs_oracle(gpu, orc):
    """Frames spanning many 4096-sample segments, every encoder, odd tails."""
    rng = np.random.default_rng(1)
    for n in (4095, 4096, 4097, 8191, 12289, 65536 + 17, 300000):
        for pre, enc, g, outl in [(1, 1, 32, 0), (0, 2, 8, 107), (1, 2, 1055, 500), (1, 1, 3, 0),
                                  (0, 0, 1, 0), (1, 1, 65535, 0), (1, 2, 1, 5)]:
            x = (np.cumsum(rng.integers(-300, 300, n)) & 0xFFFF).astype(np.uint16)
            x[rng.integers(0, n, n // 50)] = rng.integers(0, 65536, n // 50)
            outs = []
            for lib in (gpu, orc):
                ctx = api.CmpContext()
                p = api.CmpParams(primary_preprocessing=pre, primary_encoder_type=enc, primary_encoder_param=g,
                                  primary_encoder_outlier=outl, checksum_enabled=int(n % 2))
                lib.set_timestamp_func(lambda: (7, 9))
                assert not api.is_error(lib.initialise(ctx, p))
                cap = 3 * x.nbytes + 64
                dst = api.aligned_empty(cap)
                r = lib.compress_u16(ctx, dst, cap, x)
                outs.append((r, bytes(dst[:r]) if not api.is_error(r) else None))
                lib.set_timestamp_func(None)
            assert outs[0] == outs[1], (n, pre, enc, g)


@pytest.mark.parametrize("kind", scenarios.KINDS)
def test_iwt_sizes_vs_oracle(gpu, orc, kind):
    """IWT preprocessing (reference preprocess.c:140-221, 321-371) at level and
    kernel boundaries: the whole-frame LDS kernel up to 65536 samples, the
    per-level global kernels above; primary IWT with and without a MODEL
    secondary (the model overwrites the coefficients in the work buffer as
    the samples are encoded), and IWT as the secondary pass."""
    sb = 4 if kind == "i16_in_i32" else 2
    for n in (1, 2, 3, 4, 5, 6, 7, 9, 16, 17, 33, 64, 128, 192, 1000, 4095, 4096, 4097, 8256, 65472, 65535,
              65536, 65537, 131075, 300001, 1048576 + 64):
        for prm in (dict(primary_preprocessing=2, primary_encoder_type=1, primary_encoder_param=16),
                    dict(primary_preprocessing=2, primary_encoder_type=2, primary_encoder_param=10,
                         primary_encoder_outlier=200, secondary_iterations=2, secondary_preprocessing=3,
                         secondary_encoder_type=2, secondary_encoder_param=8, secondary_encoder_outlier=107,
                         model_rate=11, checksum_enabled=1),
                    dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32,
                         secondary_iterations=1, secondary_preprocessing=2, secondary_encoder_type=0)):
            if n > 70000 and prm.get("secondary_iterations") == 2:
                continue
            outs = []
            for lib in (gpu, orc):
                p = api.CmpParams(**prm)
                ctx = api.CmpContext()
                wbs = lib.cal_work_buf_size(p, n * sb)
                wb = api.aligned_empty(max(wbs, 2), fill=0x5A)
                lib.set_timestamp_func(lambda: (1, 2))
                assert not api.is_error(lib.initialise(ctx, p, wb, wbs))
                res = []
                r2 = np.random.default_rng(n)
                for step in range(3):
                    x = np.cumsum(r2.integers(-900, 900, n)) & 0xFFFF
                    x[r2.integers(0, n, max(1, n // 100))] = r2.integers(0, 65536, max(1, n // 100))
                    if kind == "i16_in_i32":
                        x = (x | (r2.integers(0, 65536, n) << 16)).astype(np.uint32).view(np.int32)
                    else:
                        x = x.astype(np.uint16) if kind == "u16" else x.astype(np.uint16).view(np.int16)
                    cap = 3 * 2 * n + 64 if step != 1 else 16 + n  # step 1: too small (fallback off)
                    dst = api.aligned_empty(cap + 64, fill=0xAB)
                    r = lib.compress(kind, ctx, dst, cap, x)
                    res.append((r, bytes(dst[:r]) if not api.is_error(r) else None, bytes(wb)))
                lib.set_timestamp_func(None)
                outs.append(res)
            assert outs[0] == outs[1], (kind, n, prm)


def test_gpu_synth_matches_oracle(eng, orc_ext):
    import torch
    for sb, W in ((2, 32), (4, 32), (2, 1024)):
        n, nf = 70000, 3
        t = torch.empty(nf * n * sb, dtype=torch.uint8, device="cuda")
        assert eng.synthesize(t.data_ptr(), sb, 0xA1A6, 5, n, nf, n * sb, W) == 0
        eng.synchronize()
        got = t.cpu().numpy()
        for f in range(nf):
            want = np.empty(n, dtype=np.uint16 if sb == 2 else np.int32)
            (orc_ext.orc_synth_u16 if sb == 2 else orc_ext.orc_synth_i32)(0xA1A6, 5 + f, n, W, want.ctypes.data)
            assert bytes(got[f * n * sb:(f + 1) * n * sb]) == want.tobytes()


@pytest.mark.parametrize("name", ["cfg1_example", "cfg2_64Mi", "cfg3_autorice", "cfg4_8192", "cfg5_model"])
def test_config_digest_gpu(gpu, eng, name):
    cfg = configs.CONFIGS[name]
    frames, gs, sz = configs.gpu_frames(gpu, eng, cfg)
    d = configs.frame_digest(frames)
    gold = CFG_GOLD[name]
    assert d["total_bytes"] == gold["total_bytes"]
    assert d["sizes_digest"] == gold["sizes_digest"]
    assert d["digest"] == gold["digest"]
    if gs is not None:
        assert hashlib.sha256(np.array(gs, dtype=np.uint32).tobytes()).hexdigest() == gold["rice_g_digest"]


def test_cfg2_roundtrip_decode(gpu, eng, orc_ext):
    """Size-independent property at full size: decode(encode(x)) == x."""
    cfg = configs.CONFIGS["cfg2_64Mi"]
    frames, _, _ = configs.gpu_frames(gpu, eng, cfg)
    data = configs.gen_inputs_cpu(orc_ext, cfg, frames=range(0, 16, 5))
    for i, f in enumerate(range(0, 16, 5)):
        out = np.zeros(cfg["n"], dtype=np.uint16)
        fr = np.frombuffer(frames[f], dtype=np.uint8)
        assert orc_ext.orc_decode(fr.ctypes.data, len(fr), None, out.ctypes.data, len(out)) == cfg["n"]
        assert np.array_equal(out, data[i])
