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


def _compare(prod, eng, orc, trial):
    params, kind, n, nctx, fpc, cap, srcs = bs.make_case(api, trial)
    want = bs.run_batch_host(orc, api, params, kind, n, nctx, fpc, cap, srcs)
    got = bs.run_batch_gpu(prod, eng, api, params, kind, n, nctx, fpc, cap, srcs)
    return got == want, want


def test_batch_vs_call_loop(prod, eng, orc):
    bad, fallbacks, errors = [], 0, 0
    for trial in range(300):
        ok, want = _compare(prod, eng, orc, trial)
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


def test_batch_fallback_identifiers(prod, eng, orc):
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
        got = bs.run_batch_gpu(prod, eng, api, params, "u16", n, nctx, fpc, cap, srcs)
        assert got == want
        assert all(r == 16 + 2 * n + 4 for r, _ in want[0])
