"""CPU: the oracle (oracle/liborc.so) against the reference's golden vectors.

Pins the CPU restatement before it is trusted as the checker for the GPU:
  - known-answer cases from the reference's own tests (tests/golden/kats.json)
  - seeded multi-frame scenario digests produced by the compiled reference
  - BASELINE config digests (small configs; large ones are GPU tests)
  - XXH32 against the published implementation (python xxhash module)
  - live oracle-vs-reference runs when oracle/_ref is built here
"""
import hashlib
import json
import os

import numpy as np
import pytest

import configs
import scenarios
from conftest import GOLDEN_DIR, load_pkg
from golden.gen_golden import run_kat

api = load_pkg().cmpapi

with open(os.path.join(GOLDEN_DIR, "kats.json")) as f:
    KATS = json.load(f)["cases"]
with open(os.path.join(GOLDEN_DIR, "random_sequences.json")) as f:
    SEQS = json.load(f)["cases"]
with open(os.path.join(GOLDEN_DIR, "configs.json")) as f:
    CFG_GOLD = json.load(f)["configs"]


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_oracle(orc, kat):
    assert run_kat(orc, kat) == kat["expected"]


def test_random_sequences_oracle(orc):
    bad = []
    for case in SEQS:
        params, kind, n = scenarios.random_case(api.CmpParams, case["trial"], allow_iwt=True)
        assert (kind, n) == (case["kind"], case["n"])
        res = scenarios.run_sequence(orc, params, kind, n, seed=case["trial"])
        if hashlib.sha256(repr(res).encode()).hexdigest() != case["digest"]:
            bad.append(case["trial"])
    assert not bad, f"oracle differs from the reference on trials {bad[:10]}"


@pytest.mark.parametrize("name", ["cfg1_example", "cfg2_64Mi", "cfg3_autorice"])
def test_config_digest_oracle(name, orc_ext):
    frames, gs = configs.cpu_frames(configs_path_orc(), orc_ext, configs.CONFIGS[name])
    d = configs.frame_digest(frames)
    gold = CFG_GOLD[name]
    assert d["total_bytes"] == gold["total_bytes"]
    assert d["sizes_digest"] == gold["sizes_digest"]
    assert d["digest"] == gold["digest"]
    if gs is not None:
        assert hashlib.sha256(np.array(gs, dtype=np.uint32).tobytes()).hexdigest() == gold["rice_g_digest"]


def configs_path_orc():
    from conftest import ORC_PATH
    return ORC_PATH


def test_xxh32_matches_published(orc_ext):
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(7)
    for ln in [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 100, 4096, 65537]:
        b = rng.integers(0, 256, ln, dtype=np.uint8)
        for seed in (0, 419764627, 0xFFFFFFFF):
            want = xxhash.xxh32_intdigest(b.tobytes(), seed=seed)
            assert orc_ext.orc_xxh32(b.ctypes.data, ln, seed) == want


def test_oracle_decoder_roundtrip(orc, orc_ext):
    rng = np.random.default_rng(3)
    for pre, enc, g in [(0, 0, 1), (1, 1, 32), (1, 1, 1055), (1, 2, 8), (0, 2, 300), (1, 1, 1)]:
        x = (np.cumsum(rng.integers(-40, 40, 5000)) & 0xFFFF).astype(np.uint16)
        x[::97] = rng.integers(0, 65536, len(x[::97]))
        ctx = api.CmpContext()
        p = api.CmpParams(primary_preprocessing=pre, primary_encoder_type=enc, primary_encoder_param=g,
                          primary_encoder_outlier=107)
        assert not api.is_error(orc.initialise(ctx, p))
        cap = orc.compress_bound(x.nbytes)
        dst = api.aligned_empty(cap)
        r = orc.compress_u16(ctx, dst, cap, x)
        assert not api.is_error(r)
        out = np.zeros_like(x)
        assert orc_ext.orc_decode(dst.ctypes.data, r, None, out.ctypes.data, len(out)) == len(x)
        assert np.array_equal(out, x)


def test_oracle_vs_reference_live(orc, ref):
    bad = []
    for trial in range(5000, 5300):
        params, kind, n = scenarios.random_case(api.CmpParams, trial, allow_iwt=True)
        if scenarios.run_sequence(orc, params, kind, n, seed=trial) != \
                scenarios.run_sequence(ref, params, kind, n, seed=trial):
            bad.append(trial)
    assert not bad
