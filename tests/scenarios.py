"""Randomised multi-frame scenarios over the cmp.h API.

`run_sequence` drives any CmpLib (GPU product, CPU oracle, compiled
reference) through cmp_initialise + several cmp_compress_* calls with the same
seeded inputs, capacities and timestamp source, and returns everything
observable: return values, frame bytes, context fields and the work buffer
(model).  Two implementations agree iff the tuples are equal.
"""
import random

import numpy as np

KINDS = ("u16", "i16", "i16_in_i32")
G_CHOICES = (1, 2, 3, 7, 8, 10, 16, 32, 100, 1055, 4096, 65535)


def make_params(P, rng, allow_iwt=True):
    pre_choices = [0, 1, 2] if allow_iwt else [0, 1]
    sec_choices = [0, 1, 2, 3] if allow_iwt else [0, 1, 3]
    return P(primary_preprocessing=rng.choice(pre_choices),
             primary_encoder_type=rng.choice([0, 1, 2]),
             primary_encoder_param=rng.choice(G_CHOICES),
             primary_encoder_outlier=rng.choice([1, 5, 42, 107, 200, 1000, 2**32 - 1]),
             secondary_iterations=rng.choice([0, 1, 3, 15]),
             secondary_preprocessing=rng.choice(sec_choices),
             secondary_encoder_type=rng.choice([0, 1, 2]),
             secondary_encoder_param=rng.choice([1, 8, 10, 32, 300]),
             secondary_encoder_outlier=rng.choice([3, 107, 500]),
             model_rate=rng.choice([0, 1, 11, 16]),
             checksum_enabled=rng.choice([0, 1]),
             uncompressed_fallback_enabled=rng.choice([0, 1]))


def make_src(kind, n, rng, spread):
    steps = np.array([rng.randint(-spread, spread) for _ in range(n)], dtype=np.int64)
    lo = np.cumsum(steps) & 0xFFFF
    if kind == "i16_in_i32":
        hi = np.array([rng.randint(0, 0xFFFF) for _ in range(n)], dtype=np.int64)
        return ((hi << 16) | lo).astype(np.uint32).view(np.int32)
    if kind == "u16":
        return lo.astype(np.uint16)
    return lo.astype(np.uint16).view(np.int16)


def run_sequence(lib, params, kind, n, seed, frames=5, ts_start=1000):
    """Init + `frames` compress calls; returns a comparable tuple."""
    from importlib import import_module
    api = import_module("airs_compression_amd.cmpapi")
    stamp = [ts_start]

    def ts():
        stamp[0] += 1
        return (stamp[0] >> 16, stamp[0] & 0xFFFF)

    lib.set_timestamp_func(ts)
    try:
        ctx = api.CmpContext()
        sample_bytes = 4 if kind == "i16_in_i32" else 2
        wbs = lib.cal_work_buf_size(params, n * sample_bytes)
        wb_len = wbs if not api.is_error(wbs) else 0
        wb = api.aligned_empty(max(wb_len, 2), fill=0)
        out = [lib.initialise(ctx, params, wb if wb_len else None, wb_len)]
        rng = random.Random(seed)
        for _ in range(frames):
            src = make_src(kind, n, rng, rng.choice([1, 4, 50, 3000, 30000]))
            bound = lib.compress_bound(2 * n)
            cap = rng.choice([bound if not api.is_error(bound) else 100000, 22 + 2 * n, 16 + 2 * n + 4,
                              30, 8 * rng.randint(1, 30)])
            dst = api.aligned_empty(cap + 64, fill=0xAB)
            r = lib.compress(kind, ctx, dst, cap, src)
            out.append((r, bytes(dst[:r]) if not api.is_error(r) else None, ctx.identifier,
                        ctx.sequence_number, ctx.model_size, bytes(wb)))
        return tuple(out)
    finally:
        lib.set_timestamp_func(None)


def random_case(P, trial, allow_iwt=True):
    rng = random.Random(trial)
    kind = rng.choice(KINDS)
    n = rng.choice([1, 2, 3, 5, 7, 8, 17, 64, 100, 333, 1000, 4095, 4097, 9000])
    return make_params(P, rng, allow_iwt), kind, n
