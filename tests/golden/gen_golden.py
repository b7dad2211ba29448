#!/usr/bin/env python3
"""Generate tests/golden/*.json from the reference compiled in oracle/_ref.

Run from the repo root in the build container (the reference sources exist
only there):  make -C oracle ref && python3 tests/golden/gen_golden.py

Outputs (data only; no reference source is copied):
  kats.json              known-answer cases transcribed from the reference's
                         own test/*.c and examples/ (inputs + the expected
                         bytes those files assert), each completed with the
                         full frame the compiled reference produced
  random_sequences.json  sha256 digests of seeded multi-frame scenarios
                         (tests/scenarios.py) as run by the reference
  configs.json           per-config frame-size totals and digests of the
                         BASELINE.json workloads (identifier bytes zeroed)
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg, REF_PATH, ORC_PATH  # noqa: E402

pkg = load_pkg()
api = pkg.cmpapi
import scenarios  # noqa: E402

I16_MIN, I16_MAX, U16_MAX = -32768, 32767, 65535


def P(**kw):
    return api.CmpParams(**kw)


# ---------------------------------------------------------------------------
# known-answer cases from the reference's own tests (file:line cited)
# each frame: (src list, expected payload bytes after the header or None)
# ---------------------------------------------------------------------------
def enc_kat(name, src_lines, enc, g, outl, data, payload, hdr_outlier):
    return dict(name=name, source=src_lines, kind="u16", cap=40,
                params=dict(primary_encoder_type=enc, primary_encoder_param=g,
                            primary_encoder_outlier=outl),
                frames=[dict(src=[d & 0xFFFF for d in data], payload=payload,
                             hdr=dict(encoder_outlier=hdr_outlier))])


ZERO, MULTI, RAW = 1, 2, 0
KATS = [
    enc_kat("golomb_zero_g1_normal", "test/test_encoder.c:143-150", ZERO, 1, 0, [-8, 7, -1, 0], "FFFF7FFF68", 16),
    enc_kat("golomb_zero_g1_lowest_outlier", "test/test_encoder.c:153-160", ZERO, 1, 0, [8], "000800", 16),
    enc_kat("golomb_zero_g1_highest_outlier", "test/test_encoder.c:163-170", ZERO, 1, 0, [I16_MIN], "7FFF80", 16),
    enc_kat("golomb_zero_g10_normal", "test/test_encoder.c:173-180", ZERO, 10, 0, [82, 4, 0], "FFFF5788", 165),
    enc_kat("golomb_zero_g10_lowest_outlier", "test/test_encoder.c:183-190", ZERO, 10, 0, [-83], "000A50", 165),
    enc_kat("golomb_zero_g10_highest_outlier", "test/test_encoder.c:193-200", ZERO, 10, 0, [I16_MIN], "0FFFF0", 165),
    enc_kat("golomb_zero_gmax", "test/test_encoder.c:203-211", ZERO, U16_MAX, 0, [0, I16_MIN], "0001400040", 0xFFFF0),
    enc_kat("golomb_multi_g1_normal", "test/test_encoder.c:214-221", MULTI, 1, 5, [0, 2], "78", 5),
    enc_kat("golomb_multi_2bit_outliers", "test/test_encoder.c:224-231", MULTI, 1, 5, [-3, 3, -4, 4], "F8F9FAFB", 5),
    enc_kat("golomb_multi_4bit_outliers", "test/test_encoder.c:234-241", MULTI, 1, 5, [-5, 10], "FC9FBC", 5),
    enc_kat("golomb_multi_16bit_outlier", "test/test_encoder.c:244-251", MULTI, 1, 5, [I16_MIN], "FFF7FFD0", 5),
    enc_kat("golomb_multi_clamp_max_normal", "test/test_encoder.c:254-261", MULTI, 1, 42, [-12], "FFFFFE", 24),
    enc_kat("golomb_multi_clamp_min_outlier", "test/test_encoder.c:264-271", MULTI, 1, 42, [12], "FFFFFF00", 24),
    enc_kat("golomb_multi_clamp_max_outlier", "test/test_encoder.c:274-281", MULTI, 1, 42, [I16_MIN], "FFFFFFFEFFE7", 24),
    enc_kat("golomb_multi_gmax_zero", "test/test_encoder.c:284-291", MULTI, U16_MAX, 2**32 - 1, [0], "0000", 0xFFFE9),
    enc_kat("golomb_multi_gmax_largest", "test/test_encoder.c:294-301", MULTI, U16_MAX, 2**32 - 1, [I16_MIN], "800000", 0xFFFE9),
    dict(name="secondary_encoder_second_pass", source="test/test_encoder.c:304-349", kind="u16", cap=26,
         params=dict(primary_encoder_type=RAW, secondary_iterations=1, secondary_encoder_type=ZERO,
                     secondary_encoder_param=10),
         frames=[dict(src=[82, 4, 0], payload="005200040000", hdr=dict(sequence_number=0)),
                 dict(src=[82, 4, 0], payload="FFFF5788", hdr=dict(sequence_number=1, encoder_outlier=165))]),
]
DIFF_SRC = [0x0001, 0x0003, 0x0000, 0xFFFF, 0x0000, 0x7FFF, 0x8000, 0xFFFB]
DIFF_EXP = "".join("%04X" % (v & 0xFFFF) for v in [1, 2, -3, -1, 1, I16_MAX, 1, 0x7FFB])
for kind in ("u16", "i16", "i16_in_i32"):
    KATS.append(dict(name="diff_preprocessing_" + kind, source="test/test_preprocessing.c:36-71", kind=kind,
                     cap=38, params=dict(primary_encoder_type=RAW, primary_preprocessing=1),
                     frames=[dict(src=DIFF_SRC, payload=DIFF_EXP)]))
for kind in ("u16", "i16"):
    KATS.append(dict(name="model_preprocessing_" + kind, source="test/test_preprocessing.c:147-178", kind=kind,
                     cap=None, work=True,
                     params=dict(primary_encoder_type=RAW, secondary_preprocessing=3, secondary_iterations=1),
                     frames=[dict(src=[0, 1, 10], payload=None),
                             dict(src=[1, 3, 5], payload="00010002FFFB", hdr=dict(sequence_number=1))]))
KATS.append(dict(name="model_preprocessing_i16_in_i32", source="test/test_preprocessing.c:181-219",
                 kind="i16_in_i32", cap=30, work=True,
                 params=dict(primary_encoder_type=RAW, secondary_preprocessing=3, secondary_iterations=1),
                 frames=[dict(src=[0, 1, 10, -4 & 0xFFFFFFFF], payload=None),
                         dict(src=[1, 3, 5, -1 & 0xFFFFFFFF], payload="00010002FFFB0003",
                              hdr=dict(sequence_number=1))]))
MODEL_CASES = {
    "u16": ([0, 2, 21, 1, U16_MAX], [1, 3, 5, U16_MAX, U16_MAX], [0] * 5,
            [0, -2, -6, -61439, (-U16_MAX) & 0xFFFF]),
    "i16": ([15, 2, 21, 0, 0, I16_MIN, I16_MAX], [-2, 3, 5, -1, 0, I16_MIN, I16_MAX], [0] * 7,
            [1, -2, -6, 1, 0, (-I16_MIN) & 0xFFFF, -I16_MAX]),
    "i16_in_i32": ([15, 2, 21, 0, 0, I16_MIN, I16_MAX], [-2, 3, 5, -1, 0, I16_MIN, I16_MAX], [0] * 7,
                   [1, -2, -6, 1, 0, (-I16_MIN) & 0xFFFF, -I16_MAX]),
}
for kind, (m1, m2, m3, exp) in MODEL_CASES.items():
    KATS.append(dict(name="model_updates_" + kind, source="test/test_preprocessing.c:222-277", kind=kind,
                     cap=None, work=True,
                     params=dict(primary_encoder_type=RAW, secondary_encoder_type=RAW, secondary_preprocessing=3,
                                 model_rate=1, secondary_iterations=2),
                     frames=[dict(src=m1, payload=None), dict(src=m2, payload=None),
                             dict(src=m3, payload="".join("%04X" % (v & 0xFFFF) for v in exp),
                                  hdr=dict(sequence_number=2, model_rate=1))]))
for kind in ("u16", "i16", "i16_in_i32"):
    KATS.append(dict(name="fallback_primary_" + kind, source="test/test_cmp.c:634-700", kind=kind, cap=26,
                     params=dict(uncompressed_fallback_enabled=1, primary_preprocessing=1,
                                 primary_encoder_type=ZERO, primary_encoder_param=1),
                     frames=[dict(src=[0xAAAA, 0xBBBB, 0xCCCC], payload="AAAABBBBCCCC",
                                  hdr=dict(preprocessing=0, encoder_type=0)),
                             dict(src=[0, 0, 0, 0], payload="AA",
                                  hdr=dict(preprocessing=1, encoder_type=1, encoder_param=1,
                                           encoder_outlier=16))]))
# IWT transform KATs (test/test_preprocessing.c:74-144): UNCOMPRESSED + IWT,
# the payload is the multi-level coefficients as big-endian int16
IWT_CASES = [([42], [42]), ([-23809, 23901], [-32722, -17826]), ([-1, 2, -3, 4, -5], [0, 4, 0, 8, -2]),
             ([0, 0, 2, 0, 0, 0, 0], [-1, -1, 2, -1, -1, 0, 1]),
             ([-3, 2, -1, 3, -2, 5, 0, 7], [0, 4, 2, 5, 1, 6, 3, 7])]
for vals, exp in IWT_CASES:
    for kind in ("u16", "i16", "i16_in_i32"):
        KATS.append(dict(name="iwt_%d_%s" % (len(vals), kind), source="test/test_preprocessing.c:74-144",
                         kind=kind, cap=None, work=True,
                         params=dict(primary_encoder_type=RAW, primary_preprocessing=2),
                         frames=[dict(src=[v & (0xFFFFFFFF if kind == "i16_in_i32" else 0xFFFF) for v in vals],
                                      payload="".join("%04X" % (v & 0xFFFF) for v in exp),
                                      hdr=dict(preprocessing=2, encoder_type=0))]))
# examples/simple_compression.c:58-322 (dummy timestamp: fine counter from 1)
EXAMPLE = dict(name="simple_compression_example", source="examples/simple_compression.c:101-296",
               kind="u16", cap="bound", work=True, timestamp="example",
               params=dict(primary_preprocessing=1, primary_encoder_type=ZERO, primary_encoder_param=1055,
                           secondary_iterations=15, secondary_preprocessing=3, secondary_encoder_type=MULTI,
                           secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11,
                           uncompressed_fallback_enabled=1, checksum_enabled=1),
               frames=[dict(src=[0, 1, 2]), dict(src=[2, 1, 1])],
               # the two frames the example prints (both fall back to raw + checksum)
               expect_frames=["825800001A000006" "0000000000040008" "000000010002" "551504C6",
                              "825800001A000006" "0000000000060008" "000200010001" "6702BD75"])
KATS.append(EXAMPLE)


def example_timestamp():
    state = [0, 0]

    def ts():
        if state[1] == 0xFFFF:
            state[0] += 1
        state[1] = (state[1] + 1) & 0xFFFF
        return (state[0], state[1])
    return ts


def src_array(kind, vals):
    if kind == "i16_in_i32":
        return np.array([v & 0xFFFFFFFF for v in vals], dtype=np.uint32).view(np.int32)
    return np.array([v & 0xFFFF for v in vals], dtype=np.uint16)


def run_kat(lib, kat):
    """Run one KAT through lib; returns list of (ret, frame_hex, ctx fields)."""
    params = P(**kat["params"])
    if kat.get("timestamp") == "example":
        lib.set_timestamp_func(example_timestamp())
    else:
        ctr = [0]

        def ts():
            ctr[0] += 1
            return (0, ctr[0])
        lib.set_timestamp_func(ts)
    try:
        ctx = api.CmpContext()
        bytes_per = 4 if kat["kind"] == "i16_in_i32" else 2
        n = len(kat["frames"][0]["src"])
        wbs = lib.cal_work_buf_size(params, n * bytes_per)
        assert not api.is_error(wbs)
        wb = api.aligned_empty(max(wbs, 2), fill=0)
        r = lib.initialise(ctx, params, wb if wbs else None, wbs)
        assert not api.is_error(r), api.error_name(r)
        out = []
        for fr in kat["frames"]:
            src = src_array(kat["kind"], fr["src"])
            cap = kat["cap"]
            if cap in (None, "bound"):
                cap = lib.compress_bound(2 * len(fr["src"]))
            dst = api.aligned_empty(cap + 16, fill=0xEE)
            r = lib.compress(kat["kind"], ctx, dst, cap, src)
            out.append(dict(ret=r, frame=bytes(dst[:r]).hex().upper() if not api.is_error(r) else None,
                            identifier=ctx.identifier, seq=ctx.sequence_number, model=bytes(wb[:wbs]).hex()))
        return out
    finally:
        lib.set_timestamp_func(None)


def check_kat_claims(kat, results):
    """Assert the expectations the reference's own test files state."""
    for i, (fr, res) in enumerate(zip(kat["frames"], results)):
        assert not api.is_error(res["ret"]), (kat["name"], i, api.error_name(res["ret"]))
        frame = bytes.fromhex(res["frame"])
        h = api.parse_header(frame)
        assert h["compressed_size"] == len(frame)
        if fr.get("payload") is not None:
            payload = frame[h["header_size"]:]
            assert payload.hex().upper() == fr["payload"], (kat["name"], i, payload.hex())
        for k, v in fr.get("hdr", {}).items():
            assert h[k] == v, (kat["name"], i, k, h[k], v)
    for i, want in enumerate(kat.get("expect_frames", [])):
        assert results[i]["frame"] == want, (kat["name"], i, results[i]["frame"])


def gen_kats(ref, orc):
    out = []
    for kat in KATS:
        res = run_kat(ref, kat)
        check_kat_claims(kat, res)
        assert run_kat(orc, kat) == res, kat["name"]
        k = dict(kat)
        k["expected"] = res
        out.append(k)
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py", produced_by="oracle/_ref/libref.so",
                       cases=out), f, indent=1)
    print("kats:", len(out))


def gen_random(ref):
    seqs = []
    for trial in range(400):
        params, kind, n = scenarios.random_case(api.CmpParams, trial, allow_iwt=True)
        res = scenarios.run_sequence(ref, params, kind, n, seed=trial)
        seqs.append(dict(trial=trial, kind=kind, n=n, params=params.as_dict(),
                         digest=hashlib.sha256(repr(res).encode()).hexdigest(),
                         ok_frames=sum(1 for x in res[1:] if not api.is_error(x[0]))))
    with open(os.path.join(HERE, "random_sequences.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py", produced_by="oracle/_ref/libref.so",
                       note="digest = sha256(repr(tests.scenarios.run_sequence(lib, ...)))", cases=seqs), f,
                  indent=0)
    print("random sequences:", len(seqs), "ok frames:", sum(s["ok_frames"] for s in seqs))


def gen_configs(only=None):
    """only: config names to regenerate (the others are kept from the file)"""
    import configs as cfgmod
    res = {}
    path = os.path.join(HERE, "configs.json")
    if only and os.path.exists(path):
        with open(path) as f:
            res = json.load(f)["configs"]
    for name in cfgmod.CONFIGS:
        if only and name not in only:
            continue
        res[name] = cfgmod.reference_digest(name, REF_PATH)
        print(name, res[name])
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py", produced_by="oracle/_ref/libref.so",
                       note="sha256 over frames in order with header identifier bytes 8..13 zeroed",
                       configs=res), f, indent=1)


def main():
    """usage: gen_golden.py [kats] [random] [configs | configs:NAME,...]   (default: all three)"""
    stages = [a for a in sys.argv[1:] if not a.startswith("-")] or ["kats", "random", "configs"]
    ref = api.CmpLib(REF_PATH)
    orc = api.CmpLib(ORC_PATH)
    if "kats" in stages:
        gen_kats(ref, orc)
    if "random" in stages:
        gen_random(ref)
    if "configs" in stages:
        gen_configs()
    for st in stages:  # configs:NAME[,NAME]: regenerate those configs only
        if st.startswith("configs:"):
            gen_configs(st.split(":", 1)[1].split(","))


if __name__ == "__main__":
    main()
