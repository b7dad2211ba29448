"""MODEL contexts in one launch (enc_walk.hip, airs_dev_walk): every
acquisition of every context in one kernel, the models kept on the chip.
cmp_gpu_compress must equal its definition, the c-major loop of
cmp_compress_* calls (include/cmp_gpu.h), run here on the oracle:
frames, sizes, context states and work buffers after the call, bit for bit.
The reference's MODEL pass and model update: lib/compress/cmp.c:120-142,
228-254, 296-311; the encoders: lib/compress/encoder.c:303-378.

Cases are built so that the walk applies (asynchronous batch: capacity at the
worst case, no fallback; n a multiple of 4096; both encoders Rice codes) and
cover: NONE/DIFF primaries, GOLOMB_ZERO and GOLOMB_MULTI on either pass
(escapes of every level, including 34-bit ones), every sample type, model
rates 0..16, checksums, several calls in a row on the same contexts (so that
contexts start mid-sequence, with their model read back from the work
buffer), and contexts whose sequences differ.  The same batches through
CMP_GPU_STEPWISE (one launch per acquisition step) must give the same bytes.
"""
import ctypes
import random

import numpy as np
import pytest

from conftest import load_pkg

pytestmark = pytest.mark.gpu
pkg = load_pkg()
api = pkg.cmpapi
P = api.CmpParams
RICE = (1, 2, 4, 8, 16, 32, 64, 1024, 32768)


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


@pytest.fixture(autouse=True)
def _engine_options(eng):
    """Engine options (cmp_gpu_engine_set_option) are per engine: every test
    leaves the module's engine at the defaults."""
    yield
    eng.set_option(pkg.OPT_WALK_SEGMENT, 0)
    eng.set_option(pkg.OPT_EXCLUSIVE, 0)


def _ts_counter(start):
    stamp = [start]

    def ts():
        stamp[0] += 1
        return (stamp[0] >> 16, stamp[0] & 0xFFFF)
    return ts


def walk_params(rng):
    return P(primary_preprocessing=rng.choice([0, 1]), primary_encoder_type=rng.choice([1, 2]),
             primary_encoder_param=rng.choice(RICE), primary_encoder_outlier=rng.choice([1, 5, 42, 107, 2**32 - 1]),
             secondary_iterations=rng.choice([1, 2, 3, 7, 15, 255]), secondary_preprocessing=3,
             secondary_encoder_type=rng.choice([1, 2]), secondary_encoder_param=rng.choice(RICE),
             secondary_encoder_outlier=rng.choice([1, 3, 107, 500, 60000]),
             model_rate=rng.choice([0, 1, 5, 11, 16]), checksum_enabled=rng.choice([0, 1]),
             uncompressed_fallback_enabled=0)


def make_frames(kind, n, count, rng):
    """Frames of a random walk plus noise; some frames are pure noise and some
    samples are outliers (every escape level of GOLOMB_MULTI)."""
    out = []
    base = np.cumsum(rng.integers(-20, 21, n))
    for _ in range(count):
        r = rng.random()
        if r < 0.15:
            v = rng.integers(-32768, 32768, n)
        else:
            v = base + rng.integers(-rng.choice([1, 8, 40, 300]), 41, n)
            hit = rng.random(n) < 0.003
            v[hit] = rng.integers(-32768, 32768, int(hit.sum()))
        v = v.astype(np.int64) & 0xFFFF
        if kind == "u16":
            out.append(v.astype(np.uint16))
        elif kind == "i16":
            out.append(v.astype(np.uint16).view(np.int16))
        else:
            out.append((v | (rng.integers(0, 0xFFFF, n) << 16)).astype(np.uint32).view(np.int32))
    return out


def _calls(nctx, calls):
    """calls: (fpc, srcs) on every context, or (c0, c1, fpc, srcs) on contexts c0 .. c1-1"""
    return [(0, nctx) + tuple(cl) if len(cl) == 2 else tuple(cl) for cl in calls]


def run_host(lib, params, kind, n, nctx, calls, cap):
    """Each call of `calls` (see _calls) compressed in order on the same contexts."""
    sb = 4 if kind == "i16_in_i32" else 2
    lib.set_timestamp_func(_ts_counter(7000))
    try:
        wbs = lib.cal_work_buf_size(params[0], n * sb)
        ctxs = [api.CmpContext() for _ in range(nctx)]
        bufs = [api.aligned_empty(wbs, fill=0) for _ in range(nctx)]
        for c in range(nctx):
            assert not api.is_error(lib.initialise(ctxs[c], params[c], bufs[c], wbs))
        out = []
        for c0, c1, fpc, srcs in _calls(nctx, calls):
            frames = []
            for c in range(c0, c1):
                for a in range(fpc):
                    dst = api.aligned_empty(cap + 64, fill=0xAB)
                    r = lib.compress(kind, ctxs[c], dst, cap, srcs[(c - c0) * fpc + a])
                    frames.append((r, bytes(dst[:r]) if not api.is_error(r) else None))
            state = [(x.identifier, x.sequence_number, x.model_size, bytes(w[:wbs])) for x, w in zip(ctxs, bufs)]
            out.append((tuple(frames), tuple(state)))
        return out
    finally:
        lib.set_timestamp_func(None)


def run_gpu(lib, eng, params, kind, n, nctx, calls, cap, flags=0):
    import torch
    sb = 4 if kind == "i16_in_i32" else 2
    stride = n * sb
    lib.set_timestamp_func(_ts_counter(7000))
    try:
        wbs = lib.cal_work_buf_size(params[0], stride)
        wstride = (wbs + 15) // 16 * 16
        work = torch.zeros(nctx * wstride, dtype=torch.uint8, device="cuda")
        ctxs = (api.CmpContext * nctx)()
        for c in range(nctx):
            assert not api.is_error(lib.initialise(ctxs[c], params[c], work.data_ptr() + c * wstride, wbs))
        out = []
        for c0, c1, fpc, srcs in _calls(nctx, calls):
            nf = (c1 - c0) * fpc
            sub = (api.CmpContext * (c1 - c0)).from_buffer(ctxs, c0 * ctypes.sizeof(api.CmpContext))
            src = torch.from_numpy(np.concatenate([np.ascontiguousarray(s).view(np.uint8) for s in srcs])).cuda()
            dstride = (cap + 64 + 7) // 8 * 8
            dst = torch.full((nf * dstride,), 0xAB, dtype=torch.uint8, device="cuda")
            sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            r = eng.compress(sub, fpc, kind, src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                             sizes.data_ptr(), flags)
            assert r == 0, api.error_name(r)
            assert eng.synchronize() == 0
            sz = sizes.cpu().numpy().astype(np.uint32)
            host = dst.cpu().numpy()
            wk = work.cpu().numpy()
            frames = tuple((int(s), bytes(host[f * dstride:f * dstride + int(s)]) if not api.is_error(int(s)) else None)
                           for f, s in enumerate(sz))
            state = tuple((ctxs[c].identifier, ctxs[c].sequence_number, ctxs[c].model_size,
                           bytes(wk[c * wstride:c * wstride + wbs])) for c in range(nctx))
            out.append((frames, state))
        return out
    finally:
        lib.set_timestamp_func(None)


def make_case(trial):
    rng = random.Random(trial)
    nrng = np.random.default_rng(trial)
    kind = rng.choice(["u16", "i16", "i16_in_i32"])
    n = 4096 * rng.choice([1, 2, 3])
    nctx = rng.choice([1, 2, 5])
    p = walk_params(rng)
    params = [p] * nctx
    ncalls = rng.choice([1, 2, 3])
    calls = []
    for _ in range(ncalls):
        fpc = rng.choice([1, 3, 8, 17])
        calls.append((fpc, make_frames(kind, n, nctx * fpc, nrng)))
    cap = 26 + 6 * n
    return params, kind, n, nctx, calls, cap


@pytest.mark.parametrize("block,seg,excl", [(b, None, b % 2) for b in range(6)] + [(b, "4096", b % 2) for b in range(3)])
def test_walk_vs_call_loop(prod, eng, orc, block, seg, excl):
    """seg: these few-context batches take 2048-sample segments (8 samples per
    lane); CMP_GPU_OPT_WALK_SEGMENT 4096 forces the 16-sample form on the same
    trials.  excl: CMP_GPU_OPT_EXCLUSIVE, under which grids that fit the CUs
    order their workgroups by block index instead of a ticket."""
    assert eng.set_option(pkg.OPT_WALK_SEGMENT, int(seg) if seg else 0) == 0
    assert eng.set_option(pkg.OPT_EXCLUSIVE, excl) == 0
    bad = []
    for trial in range(block * 12, block * 12 + 12):
        params, kind, n, nctx, calls, cap = make_case(trial)
        want = run_host(orc, params, kind, n, nctx, calls, cap)
        got = run_gpu(prod, eng, params, kind, n, nctx, calls, cap)
        if got != want:
            bad.append(trial)
    assert not bad, f"walk batch differs from the call loop on trials {bad}"


def test_walk_equals_stepwise(prod, eng):
    """The same batches with CMP_GPU_STEPWISE (one launch per acquisition
    step, the model through HBM) give the same frames and state."""
    for trial in (101, 102, 103, 104):
        params, kind, n, nctx, calls, cap = make_case(trial)
        a = run_gpu(prod, eng, params, kind, n, nctx, calls, cap)
        b = run_gpu(prod, eng, params, kind, n, nctx, calls, cap, flags=api.GPU_STEPWISE)
        assert a == b, trial


def test_walk_contexts_at_different_steps(prod, eng, orc):
    """Contexts whose sequences differ at the start of the walk call (per-
    context start sequence on the device), with identifiers that are then not
    affine in (context, acquisition): context c first compresses c frames on
    its own (one-context batches), then all contexts run one walk batch."""
    rng = np.random.default_rng(9)
    kind, n, nctx = "i16_in_i32", 8192, 4
    p = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=4,
          secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
          secondary_encoder_outlier=107, model_rate=11, checksum_enabled=1)
    params = [p] * nctx
    cap = 26 + 6 * n
    calls = [(c, c + 1, c, make_frames(kind, n, c, rng)) for c in range(1, nctx)]
    calls += [(7, make_frames(kind, n, nctx * 7, rng)), (2, make_frames(kind, n, nctx * 2, rng))]
    want = run_host(orc, params, kind, n, nctx, calls, cap)
    got = run_gpu(prod, eng, params, kind, n, nctx, calls, cap)
    assert got == want


def test_walk_many_frames_per_context(prod, eng, orc):
    """More frames per context than the walk keeps deferred epilogues for
    (AIRS_WALK_EPI_MAX = 64, enc_walk.hip): 70 acquisitions take the in-loop
    frame epilogue; 64 the deferred one; checksums and non-affine identifiers
    (contexts at different steps) on both."""
    rng = np.random.default_rng(17)
    kind, n, nctx = "i16", 4096, 2
    p = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=5,
          secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
          secondary_encoder_outlier=107, model_rate=11, checksum_enabled=1)
    params = [p] * nctx
    cap = 26 + 6 * n
    calls = [(1, 2, 1, make_frames(kind, n, 1, rng)), (70, make_frames(kind, n, nctx * 70, rng)),
             (64, make_frames(kind, n, nctx * 64, rng))]
    want = run_host(orc, params, kind, n, nctx, calls, cap)
    got = run_gpu(prod, eng, params, kind, n, nctx, calls, cap)
    assert got == want


def test_walk_cfg5_shape(prod, eng, orc, orc_ext):
    """BASELINE config 5's parameters and sample type (DIFF + ZERO g=16, then
    MODEL + MULTI g=8 o=107 rate 11, 15 secondaries) on 16 acquisitions of
    64 Ki-sample frames of 2 contexts, with the synthetic bench signal."""
    n, nctx, fpc = 65536, 2, 16
    srcs = []
    for f in range(nctx * fpc):
        x = np.empty(n, dtype=np.int32)
        orc_ext.orc_synth_i32(0xA1A9, f, n, 32, x.ctypes.data)
        srcs.append(x)
    p = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=15,
          secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
          secondary_encoder_outlier=107, model_rate=11)
    cap = 26 + 6 * n
    want = run_host(orc, [p] * nctx, "i16_in_i32", n, nctx, [(fpc, srcs)], cap)
    got = run_gpu(prod, eng, [p] * nctx, "i16_in_i32", n, nctx, [(fpc, srcs)], cap)
    assert got == want


CTX_CASES = [  # (kind, pre_p, enc_p, g_p, o_p, enc_s, g_s, o_s, iters, rate, checksum)
    ("i16_in_i32", 1, 1, 16, 0, 2, 8, 107, 15, 11, 0),  # BASELINE config 5's parameters
    ("u16", 0, 2, 64, 42, 1, 4, 0, 1, 16, 1),
    ("i16", 1, 2, 2, 107, 2, 1024, 60000, 2, 0, 0),  # 48-bit codes: two images do not fit, segment walk
    ("i16_in_i32", 0, 1, 1, 0, 1, 32768, 0, 7, 5, 1),
    ("i16", 1, 2, 16, 100, 2, 4, 30, 3, 9, 1),
]


@pytest.mark.parametrize("case,nctx,seg", [(c, 128, None) for c in range(len(CTX_CASES))] +
                         [(0, 32, None), (4, 32, None), (0, 32, "4096"), (2, 32, None)])
def test_walk_ctx_vs_call_loop(prod, eng, orc, case, nctx, seg):
    """Batches of >= 128 contexts of 64 Ki-sample frames take the context walk
    (one workgroup per context, walk_ctx_kernel); 32 contexts (configs[4]'s
    per-GPU share at N = 8) take the segment walk (walk_kernel, each
    acquisition's look-back one step late; 2048-sample segments, or 4096 with
    CMP_GPU_OPT_WALK_SEGMENT).  Frames, sizes, context states and work buffers equal the
    call loop; two calls in a row, so the second starts mid-sequence with the
    model read back from the work buffers."""
    if seg:
        assert eng.set_option(pkg.OPT_WALK_SEGMENT, int(seg)) == 0
    eng.set_option(pkg.OPT_EXCLUSIVE, 1 if nctx == 32 and case == 0 else 0)
    kind, pre, ep, gp, op, es, gs, osx, iters, rate, ck = CTX_CASES[case]
    rng = np.random.default_rng(500 + case + nctx)
    n = 65536
    p = P(primary_preprocessing=pre, primary_encoder_type=ep, primary_encoder_param=gp, primary_encoder_outlier=op,
          secondary_iterations=iters, secondary_preprocessing=3, secondary_encoder_type=es,
          secondary_encoder_param=gs, secondary_encoder_outlier=osx, model_rate=rate, checksum_enabled=ck)
    calls = [(2, make_frames(kind, n, nctx * 2, rng)), (1, make_frames(kind, n, nctx, rng))]
    cap = 26 + 6 * n
    want = run_host(orc, [p] * nctx, kind, n, nctx, calls, cap)
    got = run_gpu(prod, eng, [p] * nctx, kind, n, nctx, calls, cap)
    for ci, ((fw, sw), (fg, sg)) in enumerate(zip(want, got)):
        bad = [f for f in range(len(fw)) if fw[f] != fg[f]]
        assert not bad, f"call {ci}: frames {bad[:8]} differ"
        assert sw == sg, f"call {ci}: context states differ"


FRAME_CASES = [  # (kind, pre, enc, g, outlier, checksum, frames)
    ("u16", 1, 1, 32, 0, 0, 300),  # BASELINE configs 1/3's parameters; 300 frames: some workgroups code two
    ("i16", 0, 2, 8, 107, 1, 256),
    ("i16_in_i32", 1, 2, 4, 30, 0, 256),
    ("u16", 0, 1, 1024, 0, 1, 257),
]


@pytest.mark.parametrize("case", range(len(FRAME_CASES)))
def test_large_batches_64ki_vs_call_loop(prod, eng, orc, case):
    """Batches of >= 256 frames of 64 Ki samples without a model (cfg4's
    shape; a frame walk, one workgroup per frame, was measured slower than the
    encode kernel here and is not built): frames, sizes and the context state
    equal the call loop, identifiers included."""
    kind, pre, enc, g, outl, ck, nfr = FRAME_CASES[case]
    rng = np.random.default_rng(700 + case)
    n = 65536
    p = P(primary_preprocessing=pre, primary_encoder_type=enc, primary_encoder_param=g, primary_encoder_outlier=outl,
          checksum_enabled=ck)
    calls = [(nfr, make_frames(kind, n, nfr, rng))]
    cap = 26 + 6 * n
    want = run_host(orc, [p], kind, n, 1, calls, cap)
    got = run_gpu(prod, eng, [p], kind, n, 1, calls, cap)
    (fw, sw), (fg, sg) = want[0], got[0]
    bad = [f for f in range(nfr) if fw[f] != fg[f]]
    assert not bad, f"frames {bad[:8]} differ"
    assert sw == sg


UNIT_CASES = [  # (kind, pre, enc, g, outlier, checksum, units per frame, frames)
    ("u16", 1, 1, 32, 0, 0, 16, 40),  # BASELINE config 1's parameters, 16-unit frames: look-back across steps
    ("i16", 1, 1, 32, 0, 1, 3, 200),
    ("i16_in_i32", 0, 2, 8, 107, 0, 1, 700),  # one-unit frames: no look-back, many steps
    ("u16", 0, 2, 2, 60, 1, 5, 130),  # escapes longer than 32 bits
    ("i16", 1, 1, 2048, 0, 0, 2, 300),  # k = 11: the longest table codes
]


@pytest.mark.parametrize("case", range(len(UNIT_CASES)))
def test_whole_unit_frames_vs_call_loop(prod, eng, orc, case):
    """Frames of whole 16384-sample units without a model, from one unit to
    16 per frame, hundreds of frames (the look-back across many segments and
    frames): frames, sizes and the context state equal the call loop,
    identifiers included."""
    kind, pre, enc, g, outl, ck, upf, nfr = UNIT_CASES[case]
    rng = np.random.default_rng(900 + case)
    n = 16384 * upf
    p = P(primary_preprocessing=pre, primary_encoder_type=enc, primary_encoder_param=g, primary_encoder_outlier=outl,
          checksum_enabled=ck)
    calls = [(nfr, make_frames(kind, n, nfr, rng))]
    cap = 26 + 6 * n
    want = run_host(orc, [p], kind, n, 1, calls, cap)
    got = run_gpu(prod, eng, [p], kind, n, 1, calls, cap)
    (fw, sw), (fg, sg) = want[0], got[0]
    bad = [f for f in range(nfr) if fw[f] != fg[f]]
    assert not bad, f"frames {bad[:8]} differ"
    assert sw == sg


@pytest.mark.parametrize("seg", [None, "2048"])
def test_segment_walk_more_workgroups_than_resident(prod, eng, orc, seg):
    """a segment walk whose grid exceeds what the GPU holds at once
    (1100 contexts x one 4096-sample segment, 320-thread workgroups with two
    images each: at most 1024 resident; or x two 2048-sample segments, 2200
    workgroups, at most 1280 resident) and a long walk (12 acquisitions): the
    workgroups take logical indices from a ticket, so a look-back only waits
    on a running workgroup; no give-up, frames and state equal the call loop."""
    if seg:
        assert eng.set_option(pkg.OPT_WALK_SEGMENT, int(seg)) == 0
    eng.set_option(pkg.OPT_EXCLUSIVE, 1)  # too many workgroups for the direct form: the ticket anyway
    rng = np.random.default_rng(31)
    kind, n, nctx, fpc = "u16", 4096, 1100, 12
    p = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=15,
          secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
          secondary_encoder_outlier=107, model_rate=11, checksum_enabled=1)
    calls = [(fpc, make_frames(kind, n, nctx * fpc, rng))]
    cap = 26 + 6 * n
    want = run_host(orc, [p] * nctx, kind, n, nctx, calls, cap)
    got = run_gpu(prod, eng, [p] * nctx, kind, n, nctx, calls, cap)
    (fw, sw), (fg, sg) = want[0], got[0]
    bad = [f for f in range(len(fw)) if fw[f] != fg[f]]
    assert not bad, f"frames {bad[:8]} differ"
    assert sw == sg


def test_segment_walk_beside_other_kernels(prod, eng, orc, orc_ext):
    """a cfg5s8-shaped segment walk (configs[4]'s parameters, 32
    streams x 16 acquisitions x 64 Ki i16-in-i32 samples, 1024 workgroups)
    while kernels on a second stream keep the CUs busy.  The engine is not
    marked exclusive, so every workgroup numbers itself with a ticket as it
    starts and a look-back only waits on a running workgroup: bit-exact
    frames and state against the call loop, no look-back give-up
    (CMP_ERR_INT_BITSTREAM from cmp_gpu_synchronize)."""
    import threading

    import torch
    n, nctx, fpc = 65536, 32, 16
    srcs = []
    for f in range(nctx * fpc):
        x = np.empty(n, dtype=np.int32)
        orc_ext.orc_synth_i32(0xA1A9, f, n, 32, x.ctypes.data)
        srcs.append(x)
    p = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16, secondary_iterations=15,
          secondary_preprocessing=3, secondary_encoder_type=2, secondary_encoder_param=8,
          secondary_encoder_outlier=107, model_rate=11)
    cap = 26 + 6 * n
    want = run_host(orc, [p] * nctx, "i16_in_i32", n, nctx, [(fpc, srcs)], cap)
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
        got = run_gpu(prod, eng, [p] * nctx, "i16_in_i32", n, nctx, [(fpc, srcs)], cap)
    finally:
        stop.set()
        t.join()
    assert got == want
