"""cmp_gpu_compress against its definition (include/cmp_gpu.h): the c-major
loop of cmp_compress_* calls, run here on the oracle.  Cases mix uncompressed
fallback (reference cmp.c:342-393), capacities below the worst case (frames
that fail, and frames rejected before encoding), several contexts, secondary
passes and MODEL state.  Bit-exact: frames, sizes or error values, context
state and work buffers."""
import pytest

import batch_scenarios as bs
from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine()
    yield e
    e.close()


@pytest.fixture(params=["device", "host"])
def exact_mode(request):
    """Batch flags: batches that can fall back or fail run the context state
    machine on the GPU (batch_device_exact) unless CMP_GPU_HOST_STEPPED selects
    the host-stepped path (batch_exact); both must equal the call loop."""
    return api.GPU_HOST_STEPPED if request.param == "host" else 0


def _compare(prod, eng, orc, trial, flags):
    params, kind, n, nctx, fpc, cap, srcs = bs.make_case(api, trial)
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs)
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs, flags=flags)
    return got == want, want


def test_batch_vs_call_loop(prod, eng, orc, exact_mode):
    bad, fallbacks, errors = [], 0, 0
    for trial in range(300):
        ok, want = _compare(prod, eng, orc, trial, exact_mode)
        frames = want[0]
        errors += sum(api.is_error(r) for r, _ in frames)
        params = bs.make_case(api, trial)[0]
        if params.primary_encoder_type != api.ENCODER_UNCOMPRESSED:
            fallbacks += sum(1 for r, b in frames if b is not None and
                             api.parse_header(b)["encoder_type"] == api.ENCODER_UNCOMPRESSED)
        if not ok:
            bad.append(trial)
    assert not bad, f"batch differs from the call loop on trials {bad[:10]}"
    # the cases must actually exercise the failure paths
    assert errors > 50 and fallbacks > 50, (errors, fallbacks)


@pytest.mark.parametrize("n,sec,spre", [(65536, 0, 1), (65536, 2, 2), (262144, 1, 2), (4160, 2, 3)])
def test_batch_iwt_fallback_vs_call_loop(prod, eng, orc, exact_mode, n, sec, spre):
    """IWT passes with the uncompressed fallback (round 5: the device exact
    mode takes them; every IWT kernel form: the register kernel at 64 Ki,
    the two-phase kernel above, the LDS frame kernel at 4160).  Smooth frames
    compress, noise frames fall back, so the pass schedule of each context
    changes mid-batch; frames, sizes and work buffers (the coefficients, or
    the model) equal the call loop's."""
    import numpy as np
    P = api.CmpParams
    rng = np.random.default_rng(n + sec)
    params = P(primary_preprocessing=api.PREPROCESS_IWT, primary_encoder_type=1, primary_encoder_param=4,
               secondary_iterations=sec, secondary_preprocessing=spre, secondary_encoder_type=1,
               secondary_encoder_param=8, checksum_enabled=1, uncompressed_fallback_enabled=1, model_rate=5)
    nctx, fpc = 3, 5
    t = np.arange(n)
    srcs = []
    for f in range(nctx * fpc):
        if rng.random() < 0.35:
            srcs.append(rng.integers(0, 65536, n).astype(np.uint16))
        else:
            srcs.append((30000 + 8000 * np.sin(t / (50.0 + 7 * f)) + rng.integers(-20, 21, n)).astype(np.uint16))
    cap = 16 + 2 * n + 4
    want = bs.run_batch_host(orc, api, params, "u16", n, nctx, fpc, cap, srcs)
    got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, nctx, fpc, cap, srcs, flags=exact_mode)
    assert got == want
    frames = want[0]
    raw = sum(1 for r, b in frames if b is not None and api.parse_header(b)["encoder_type"] == api.ENCODER_UNCOMPRESSED)
    assert 0 < raw < len(frames), raw


def test_batch_fallback_identifiers(prod, eng, orc, exact_mode):
    """Noise frames that do not compress: every frame falls back; identifiers
    advance by three draws per primary fallback and two per secondary one."""
    import numpy as np
    P = api.CmpParams
    rng = np.random.default_rng(5)
    for sec in (0, 2):
        params = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=2,
                   secondary_iterations=sec, secondary_preprocessing=1, secondary_encoder_type=1,
                   secondary_encoder_param=2, checksum_enabled=1, uncompressed_fallback_enabled=1)
        n, nctx, fpc = 3000, 3, 4
        srcs = [rng.integers(0, 65536, n).astype(np.uint16) for _ in range(nctx * fpc)]
        cap = 26 + 6 * n
        want = bs.run_batch_host(orc, api, params, "u16", n, nctx, fpc, cap, srcs)
        got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, nctx, fpc, cap, srcs, flags=exact_mode)
        assert got == want
        assert all(r == 16 + 2 * n + 4 for r, _ in want[0])


def test_batch_size_field_overflow_vs_call_loop(prod, eng, orc, exact_mode):
    """4 Mi-sample frames whose worst case exceeds the 24-bit compressed-size
    field: noise frames fail with HDR_CMP_SIZE_TOO_LARGE even though the
    capacity holds the worst case, and the reference then does not advance
    the sequence number (cmp.c:321-338), so with secondary passes the next
    frame's pass depends on the failure (the batch must take the
    step-by-step path here)."""
    import numpy as np
    P = api.CmpParams
    rng = np.random.default_rng(11)
    n, nctx, fpc = 4 << 20, 2, 3
    params = P(primary_preprocessing=0, primary_encoder_type=2, primary_encoder_param=1,
               primary_encoder_outlier=24, secondary_iterations=2, secondary_preprocessing=0,
               secondary_encoder_type=2, secondary_encoder_param=1, secondary_encoder_outlier=24)
    noise = rng.integers(0, 65536, n).astype(np.uint16)   # ~48 bits/sample: > 2^24 - 1 bytes
    quiet = np.zeros(n, dtype=np.uint16)
    srcs = [noise, quiet, quiet, quiet, noise, quiet]
    cap = 26 + 6 * n
    want = bs.run_batch_host(orc, api, params, "u16", n, nctx, fpc, cap, srcs)
    assert api.error_name(want[0][0][0]) == "HDR_CMP_SIZE_TOO_LARGE", want[0][0][0]
    got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, nctx, fpc, cap, srcs, flags=exact_mode)
    assert got == want


@pytest.mark.parametrize("kind", ["i16_in_i32", "u16"])
def test_batch_model_fallback_cfg5_shape(prod, eng, orc, exact_mode, kind):
    """BASELINE config 5's parameters (DIFF + ZERO g=16, then 15 MODEL + MULTI
    passes g=8 o=107 rate 11) with the uncompressed fallback and checksums on:
    noise frames at scattered acquisition steps fall back (primary and
    secondary), so contexts drift apart in their pass sequence.  Frames,
    sizes, context states and work buffers equal the oracle's call loop."""
    import numpy as np
    P = api.CmpParams
    params = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
               secondary_iterations=15, secondary_preprocessing=3, secondary_encoder_type=2,
               secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11,
               checksum_enabled=1, uncompressed_fallback_enabled=1)
    rng = np.random.default_rng(55)
    n, nctx, fpc = 8192 + 77, 12, 16
    srcs = []
    for c in range(nctx):
        base = np.cumsum(rng.integers(-3, 4, n))
        for a in range(fpc):
            if rng.random() < 0.15:
                v = rng.integers(-32768, 32768, n)  # noise: the frame falls back
            else:
                v = base + rng.integers(-4, 5, n)
            v = v.astype(np.int64)
            if kind == "u16":
                srcs.append((v & 0xFFFF).astype(np.uint16))
            else:
                srcs.append(((v & 0xFFFF) | (rng.integers(-5, 5, n) << 16)).astype(np.int32))
    cap = 26 + 6 * n
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs)
    nfb = sum(1 for r, b in want[0] if b is not None and api.parse_header(b)["encoder_type"] == 0)
    assert nfb > 10, nfb
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs, flags=exact_mode)
    assert got == want


@pytest.mark.parametrize("kind", ["i16_in_i32", "u16"])
@pytest.mark.parametrize("flags", [0, api.GPU_STEPWISE], ids=["walk", "stepwise"])
def test_batch_walk_fallback_cfg5_shape(prod, eng, orc, kind, flags):
    """BASELINE config 5's shape with the uncompressed fallback (cfg5fb):
    128 contexts of 64 Ki-sample frames, so the batch takes the context walk
    with the fallback resolved on the chip (flags 0: one launch, the frame that
    does not fit its raw size is written raw, the model takes its samples, the
    context continues at sequence number 1; then the host draws the
    identifiers from the reported draw counts), against the per-acquisition
    device state machine (CMP_GPU_STEPWISE) and the oracle's call loop.  Noise
    frames at scattered steps fall back as primary and as secondary passes;
    two calls on the same contexts, so the second starts from contexts in
    different states.  Frames with identifiers unmasked, sizes, context
    states and work buffers."""
    import numpy as np
    P = api.CmpParams
    params = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
               secondary_iterations=15, secondary_preprocessing=3, secondary_encoder_type=2,
               secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11,
               checksum_enabled=1, uncompressed_fallback_enabled=1)
    rng = np.random.default_rng(66 + len(kind))
    n, nctx, fpc = 65536, 128, 5
    srcs = []
    for c in range(nctx):
        base = np.cumsum(rng.integers(-3, 4, n))
        for a in range(fpc):
            if rng.random() < 0.12:
                v = rng.integers(-32768, 32768, n)  # noise: the frame falls back
            else:
                v = base + rng.integers(-4, 5, n)
            v = v.astype(np.int64)
            if kind == "u16":
                srcs.append((v & 0xFFFF).astype(np.uint16))
            else:
                srcs.append(((v & 0xFFFF) | (rng.integers(-5, 5, n) << 16)).astype(np.int32))
    cap = 26 + 6 * n
    splits = [2, 3]
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs, splits=splits)
    heads = [api.parse_header(b) for r, b in want[0] if b is not None]
    nfb = sum(1 for h in heads if h["encoder_type"] == 0)
    assert nfb > 30, nfb
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs, flags=flags, splits=splits)
    assert got[1] == want[1], "context states or work buffers differ"
    bad = [f for f in range(nctx * fpc) if got[0][f] != want[0][f]]
    assert not bad, f"frames {bad[:8]} differ"


@pytest.mark.parametrize("kind,n,nctx,p_noise,sep", [("i16_in_i32", 65536, 32, 0.12, False),
                                                      ("u16", 65536, 32, 0.0, False),
                                                      ("u16", 16384, 8, 0.2, False),
                                                      ("i16_in_i32", 8192, 3, 0.3, False),
                                                      ("u16", 16384, 6, 0.25, True)])
def test_batch_segment_walk_fallback(prod, eng, orc, kind, n, nctx, p_noise, sep):
    """The fallback with too few contexts (or frames of another size) for the
    context walk: the segment walk codes every frame with the raw frame size as
    capacity; contexts with a frame that does not fit run again on the
    per-acquisition device state machine from their models as they were before
    the call (batch_walk_spec).  32 contexts of 64 Ki samples is rank 0's shard
    of config 5 at N = 8 (cfg5fbs8); p_noise 0: no frame falls back (the
    speculative walk's output stands); sep: work buffers in separate
    allocations (a model pointer per context, saved and restored one by one).
    Two calls on the same contexts.
    Frames with identifiers unmasked, sizes, context states and work buffers
    against the oracle's call loop."""
    import numpy as np
    P = api.CmpParams
    params = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
               secondary_iterations=15, secondary_preprocessing=3, secondary_encoder_type=2,
               secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11,
               checksum_enabled=1, uncompressed_fallback_enabled=1)
    rng = np.random.default_rng(n + nctx)
    fpc = 5
    srcs = []
    for c in range(nctx):
        base = np.cumsum(rng.integers(-3, 4, n))
        for a in range(fpc):
            if rng.random() < p_noise:
                v = rng.integers(-32768, 32768, n)  # noise: the frame falls back
            else:
                v = base + rng.integers(-4, 5, n)
            v = v.astype(np.int64)
            if kind == "u16":
                srcs.append((v & 0xFFFF).astype(np.uint16))
            else:
                srcs.append(((v & 0xFFFF) | (rng.integers(-5, 5, n) << 16)).astype(np.int32))
    cap = 26 + 6 * n
    splits = [2, 3]
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs, splits=splits)
    heads = [api.parse_header(b) for r, b in want[0] if b is not None]
    nfb = sum(1 for h in heads if h["encoder_type"] == 0)
    assert (nfb > 0) == (p_noise > 0), nfb
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs, splits=splits, separate_work=sep)
    assert got[1] == want[1], "context states or work buffers differ"
    bad = [f for f in range(nctx * fpc) if got[0][f] != want[0][f]]
    assert not bad, f"frames {bad[:8]} differ"


@pytest.mark.parametrize("knob", ["AIRS_TEST_COMMIT_TICKS", "AIRS_TEST_COMMIT_POLLS"])
def test_batch_commit_give_up_paths(prod, orc, knob):
    """the speculative segment walk's commit handshake when
    one side gives up waiting.  AIRS_TEST_COMMIT_TICKS=0: the commit kernel
    stops waiting for the host's release at once (as if the host thread had
    been descheduled for a second); AIRS_TEST_COMMIT_POLLS=0: the host stops
    waiting for the kernel's signal at once (as if earlier work still held the
    stream) and releases without identifiers.  Either way the headers must
    still carry the identifiers (the host patches them when the kernel's
    acknowledgement says it did not): frames with identifiers unmasked,
    sizes and context states against the oracle's call loop."""
    import os

    import numpy as np
    import torch
    P = api.CmpParams
    params = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
               secondary_iterations=15, secondary_preprocessing=3, secondary_encoder_type=2,
               secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11,
               checksum_enabled=1, uncompressed_fallback_enabled=1)
    rng = np.random.default_rng(404)
    n, nctx, fpc = 16384, 8, 5
    srcs = []
    for c in range(nctx):
        base = np.cumsum(rng.integers(-3, 4, n))
        for a in range(fpc):
            v = (base + rng.integers(-4, 5, n)).astype(np.int64)  # nothing falls back: the kernel patches
            srcs.append((v & 0xFFFF).astype(np.uint16))
    cap = 26 + 6 * n
    want = bs.run_batch_host(orc, api, params, "u16", n, nctx, fpc, cap, srcs, splits=[2, 3])
    os.environ[knob] = "0"
    try:
        e = prod.engine(torch.cuda.current_stream().cuda_stream)  # reads the knob at creation
    finally:
        del os.environ[knob]
    try:
        got = bs.run_batch_gpu(prod, e, api, params, "u16", n, nctx, fpc, cap, srcs, splits=[2, 3])
    finally:
        e.close()
    assert got[1] == want[1], "context states or work buffers differ"
    bad = [f for f in range(nctx * fpc) if got[0][f] != want[0][f]]
    assert not bad, f"frames {bad[:8]} differ"


def test_batch_mixed_fallback_model_contexts(prod, eng, orc):
    """contexts with and without the uncompressed fallback
    in one batch (different parameters: the host-stepped path), with
    dst_capacity equal to the raw frame size so that both kinds share that
    capacity.  A MODEL secondary frame that runs out of room stops updating the
    model at the failing sample when its context cannot fall back
    (cmp.c:296-311), and is replaced by a raw frame (whole model) when it
    can.  Frames, context states and work buffers equal the call loop."""
    import numpy as np
    P = api.CmpParams
    base = dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=16,
                secondary_iterations=5, secondary_preprocessing=3, secondary_encoder_type=2,
                secondary_encoder_param=8, secondary_encoder_outlier=107, model_rate=11)
    rng = np.random.default_rng(77)
    n, nctx, fpc = 5000, 4, 6
    params = [P(**base, uncompressed_fallback_enabled=c % 2) for c in range(nctx)]
    srcs = []
    for c in range(nctx):
        walk = np.cumsum(rng.integers(-3, 4, n))
        for a in range(fpc):
            v = rng.integers(-32768, 32768, n) if (c + a) % 3 == 2 else walk + rng.integers(-4, 5, n)
            srcs.append((v.astype(np.int64) & 0xFFFF).astype(np.uint16))
    cap = 16 + 2 * n  # the raw frame size: what fallback contexts use as first-attempt capacity
    want = bs.run_batch_host(orc, api, params, "u16", n, nctx, fpc, cap, srcs)
    assert sum(api.is_error(r) for r, _ in want[0]) > 2  # fallback-less contexts fail
    got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, nctx, fpc, cap, srcs)
    assert got == want


def test_batch_rejects_overlapping_frames(prod, eng):
    import torch
    n = 4096
    src = torch.zeros(2 * n * 2, dtype=torch.uint8, device="cuda")
    cap = prod.compress_bound(2 * n)
    dst = torch.zeros(4 * cap, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(2, dtype=torch.int32, device="cuda")
    ctxs = (api.CmpContext * 1)()
    assert not api.is_error(prod.initialise(ctxs[0], api.CmpParams(primary_preprocessing=1,
                                                                   primary_encoder_type=1,
                                                                   primary_encoder_param=4)))
    # dst_stride below the capacity, then src_stride below the frame size
    assert api.is_error(eng.compress(ctxs, 2, "u16", src.data_ptr(), 2 * n, 2 * n, dst.data_ptr(), 64, cap,
                                     sizes.data_ptr()))
    assert api.is_error(eng.compress(ctxs, 2, "u16", src.data_ptr(), 2 * n - 2, 2 * n, dst.data_ptr(),
                                     (cap + 7) // 8 * 8, cap, sizes.data_ptr()))
    assert eng.compress(ctxs, 2, "u16", src.data_ptr(), 2 * n, 2 * n, dst.data_ptr(), (cap + 7) // 8 * 8, cap,
                        sizes.data_ptr()) == 0
    assert eng.synchronize() == 0


def test_host_api_one_context_per_thread(prod, orc):
    """cmp_compress_* from several threads, one context each (the reference's
    threading model): every frame equals the oracle's frame for the
    same context sequence.  Identifier bytes are masked: the threads draw
    from one shared counter in a nondeterministic order."""
    import threading
    import numpy as np
    P = api.CmpParams
    nthreads, frames_per_thread = 8, 12
    params = [P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=1 << (t % 7),
                secondary_iterations=3 if t % 2 else 0, secondary_preprocessing=1, secondary_encoder_type=2,
                secondary_encoder_param=3 + t, secondary_encoder_outlier=40, checksum_enabled=t % 3 == 0)
              for t in range(nthreads)]
    rng = np.random.default_rng(3)
    inputs = [[(np.cumsum(rng.integers(-20, 21, 3000 + 97 * t)) & 0xFFFF).astype(np.uint16)
               for _ in range(frames_per_thread)] for t in range(nthreads)]

    def run(lib, t, out):
        ctx = api.CmpContext()
        assert not api.is_error(lib.initialise(ctx, params[t]))
        for x in inputs[t]:
            cap = lib.compress_bound(x.nbytes)
            dst = api.aligned_empty(cap)
            r = lib.compress_u16(ctx, dst, cap, x)
            b = bytearray(dst[:r]) if not api.is_error(r) else None
            if b is not None:
                b[8:14] = b"\0" * 6
            out.append((r, bytes(b) if b is not None else None))

    want = []
    for t in range(nthreads):
        w = []
        run(orc, t, w)
        want.append(w)
    got = [[] for _ in range(nthreads)]
    errs = []

    def worker(t):
        try:
            run(prod, t, got[t])
        except Exception as e:  # reported below
            errs.append(repr(e))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=120)
    assert not errs, errs
    for t in range(nthreads):
        assert got[t] == want[t], f"thread {t} differs from the oracle"
