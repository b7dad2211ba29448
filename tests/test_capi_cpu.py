"""CPU: the product C-ABI library loads, exports every declared symbol, and
its host-side logic (validation, bounds, context state, errors) matches the
oracle.  No compute call is made here (there is no GPU in this container)."""
import ctypes
import os
import random
import re

import pytest

import scenarios
from conftest import ROOT, load_pkg

api = load_pkg().cmpapi


def declared_functions():
    names = set()
    for h in ("cmp.h", "cmp_errors.h", "cmp_gpu.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b([a-z_0-9]+)\s*\(", text):
            if m.group(1).startswith("cmp_") and not m.group(1).isupper():
                names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol(prod):
    names = declared_functions()
    assert "cmp_compress_u16" in names and "cmp_gpu_compress" in names
    missing = [n for n in names if not hasattr(prod.lib, n)]
    assert not missing


def test_struct_layout_matches_reference_abi():
    assert ctypes.sizeof(api.CmpParams) == 44
    assert ctypes.sizeof(api.CmpContext) == 80
    assert api.CmpContext.work_buf.offset == 48
    assert api.CmpContext.identifier.offset == 64
    assert api.CmpContext.sequence_number.offset == 72


def test_bounds_and_work_buffer_sizes_match_oracle(prod, orc):
    for size in [0, 1, 2, 3, 100, 2**16, 2796190, 2796192, 2**24 - 1, 2**24, 2**32 - 1]:
        assert prod.compress_bound(size) == orc.compress_bound(size), size
    rng = random.Random(11)
    for _ in range(300):
        p = scenarios.make_params(api.CmpParams, rng)
        p.primary_preprocessing = rng.choice([0, 1, 2, 3, 7])
        p.secondary_preprocessing = rng.choice([0, 1, 2, 3, 9])
        for size in (0, 1, 7, 4096):
            assert prod.cal_work_buf_size(p, size) == orc.cal_work_buf_size(p, size)
    assert prod.cal_work_buf_size(None, 4) == orc.cal_work_buf_size(None, 4)


def test_initialise_validation_matches_oracle(prod, orc):
    rng = random.Random(5)
    for _ in range(2000):
        p = scenarios.make_params(api.CmpParams, rng)
        p.primary_encoder_param = rng.choice([0, 1, 2, 65535, 65536, 2**32 - 1])
        p.secondary_encoder_param = rng.choice([0, 1, 8, 65536])
        p.primary_encoder_outlier = rng.choice([0, 1, 23, 24, 25, 2**32 - 1])
        p.secondary_iterations = rng.choice([0, 1, 255, 256])
        p.model_rate = rng.choice([0, 16, 17])
        p.primary_encoder_type = rng.choice([0, 1, 2, 3])
        wb = rng.choice([None, 2, 3])
        size = rng.choice([0, 2, 2**32 - 1, 2**32 - 200])
        buf = api.aligned_empty(16)
        ptr = None if wb is None else buf.ctypes.data + (wb - 2)
        results = []
        for lib in (prod, orc):
            ctx = api.CmpContext()
            results.append((lib.initialise(ctx, p, ptr, size), ctx.magic, ctx.sequence_number,
                            ctx.work_buf_size))
        assert results[0] == results[1]


def test_compress_argument_errors_without_gpu(prod, orc):
    """Errors detected before any device work are identical on CPU."""
    p = api.CmpParams(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=8)
    src = api.aligned_empty(64, fill=1)
    dst = api.aligned_empty(256)
    for lib in (prod, orc):
        ctx = api.CmpContext()
        assert not api.is_error(lib.initialise(ctx, p))
    cases = [
        lambda L, c: L.compress_u16(c, dst, 256, None, 64),
        lambda L, c: L.compress_u16(c, dst, 256, src, 0),
        lambda L, c: L.compress_i16_in_i32(c, dst, 256, src, 6),
        lambda L, c: L.compress_u16(None, dst, 256, src, 64),
        lambda L, c: L.compress_u16(c, dst, 2**32 - 1, src, 64),
        lambda L, c: L.compress_u16(c, None, 256, src, 64),
        lambda L, c: L.compress_u16(c, dst.ctypes.data + 4, 256, src, 64),
        lambda L, c: L.compress_u16(c, dst, 10, src, 64),
        lambda L, c: L.compress_u16(c, dst, 256, src, 2**24),
    ]
    for i, case in enumerate(cases):
        outs = []
        for lib in (prod, orc):
            ctx = api.CmpContext()
            lib.initialise(ctx, p)
            outs.append((case(lib, ctx), ctx.sequence_number))
        assert outs[0] == outs[1], i
    # uninitialised context
    for lib in (prod, orc):
        assert api.error_name(lib.compress_u16(api.CmpContext(), dst, 256, src, 64)) == "CONTEXT_INVALID"
        assert api.error_name(lib.reset(api.CmpContext())) == "CONTEXT_INVALID"


def test_error_strings_match_oracle(prod, orc):
    for code in list(api.ERR.values()) + [2, 99, 127, 129]:
        assert prod.get_error_string(code) == orc.get_error_string(code)
        v = (-code) & 0xFFFFFFFF
        assert prod.get_error_message(v) == orc.get_error_message(v)
        assert prod.get_error_code(v) == orc.get_error_code(v)
        assert prod.is_error(v) == orc.is_error(v)


def test_timestamp_identifiers_match_oracle(prod, orc):
    p = api.CmpParams()
    for lib in (prod, orc):
        vals = iter([(0x1234, 0x5678), (1, 2), (0xFFFFFFFF, 0xFFFF)])
        lib.set_timestamp_func(lambda: next(vals))
        ctx = api.CmpContext()
        assert not api.is_error(lib.initialise(ctx, p))
        assert ctx.identifier == 0x12345678
        assert not api.is_error(lib.reset(ctx))
        assert ctx.identifier == (1 << 16) | 2
        lib.reset(ctx)
        assert ctx.identifier == 0xFFFFFFFFFFFF
        lib.set_timestamp_func(None)


def test_compress_without_gpu_fails_loudly(prod, capfd):
    if prod.gpu_available():
        pytest.skip("GPU present")
    p = api.CmpParams(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=8)
    ctx = api.CmpContext()
    assert not api.is_error(prod.initialise(ctx, p))
    src = api.aligned_empty(64, fill=1)
    dst = api.aligned_empty(256)
    r = prod.compress_u16(ctx, dst, 256, src, 64)
    assert api.error_name(r) == "GENERIC"
    assert "no usable GPU" in capfd.readouterr().err
