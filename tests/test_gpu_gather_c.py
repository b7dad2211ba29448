"""cmp_gpu_gather (the C multi-GPU gather over RCCL, csrc/cmp_gather.c) on the
box's one GPU: a one-rank RCCL communicator made here through librccl, frames
compressed by cmp_gpu_compress with their identifier draws reported, gathered
to rank 0 in global order with the identifiers patched; checked byte for byte
against the frames themselves and the identifiers one process draws
(base + the inclusive scan of the draws, shard.py assign_identifiers).  The
all-gather, the packing, the grouped transfers and the patch kernel all run;
the multi-rank exchange itself needs several GPUs (the plan's logic for any
number of ranks is tests/test_gather_plan.py)."""
import ctypes

import numpy as np
import pytest

from conftest import load_pkg

pytestmark = pytest.mark.gpu
pkg = load_pkg()
api = pkg.cmpapi


class _UID(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


@pytest.fixture(scope="module")
def comm():
    import torch
    torch.cuda.init()
    R = ctypes.CDLL("librccl.so.1", mode=ctypes.RTLD_GLOBAL)
    uid = _UID()
    assert R.ncclGetUniqueId(ctypes.byref(uid)) == 0
    c = ctypes.c_void_p()
    R.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UID, ctypes.c_int]
    assert R.ncclCommInitRank(ctypes.byref(c), 1, uid, 0) == 0
    yield c.value
    R.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    R.ncclCommDestroy(c)


@pytest.fixture(scope="module")
def eng(prod):
    import torch
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine(torch.cuda.current_stream().cuda_stream)
    yield e
    e.close()


def _compress(prod, eng, nctx, fpc, n, secondary):
    import torch
    P = api.CmpParams
    prm = P(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32,
            secondary_iterations=secondary, secondary_preprocessing=1, secondary_encoder_type=1,
            secondary_encoder_param=16, checksum_enabled=1)
    nf = nctx * fpc
    src = torch.empty(nf * 2 * n, dtype=torch.uint8, device="cuda")
    assert eng.synthesize(src.data_ptr(), 2, 0xA1A8, 0, n, nf, 2 * n, 32) == 0
    cap = prod.compress_bound(2 * n)
    dstride = (cap + 7) // 8 * 8
    dst = torch.zeros(nf * dstride, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = pkg.context_array(nctx)
    for c in range(nctx):
        assert not api.is_error(prod.initialise(ctxs[c], prm))
    draws = np.zeros(nf, dtype=np.uint8)
    assert eng.compress(ctxs, fpc, "u16", src.data_ptr(), 2 * n, 2 * n, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr(), 0, draws.ctypes.data) == 0
    assert eng.synchronize() == 0
    return dst, dstride, cap, sizes, draws


@pytest.mark.parametrize("layout,nctx,fpc,secondary", [("roundrobin", 1, 12, 0), ("block", 3, 4, 0),
                                                       ("streams", 4, 5, 3)])
def test_gather_one_rank(prod, eng, comm, layout, nctx, fpc, secondary):
    import torch
    n = 65536
    dst, dstride, cap, sizes, draws = _compress(prod, eng, nctx, fpc, n, secondary)
    nf = nctx * fpc
    lay = {"roundrobin": pkg.LAYOUT_ROUNDROBIN, "block": pkg.LAYOUT_BLOCK, "streams": pkg.LAYOUT_STREAMS}[layout]
    gfpc = fpc if layout == "streams" else 1
    sz = sizes.cpu().numpy().astype(np.int64)
    total = int(sum((s + 7) // 8 * 8 for s in sz))
    out = torch.full((total + 64,), 0xCD, dtype=torch.uint8, device="cuda")
    offs = np.zeros(nf, dtype=np.uint64)
    osz = np.zeros(nf, dtype=np.uint32)
    base = 5000
    r = eng.gather(comm, 0, lay, gfpc, dst.data_ptr(), dstride, cap, sizes.data_ptr(), draws.ctypes.data, nf,
                   out.data_ptr(), out.numel(), offs.ctypes.data, osz.ctypes.data, base, pkg.GATHER_PATCH_IDS)
    assert r == 0, api.error_name(r)
    assert eng.synchronize() == 0
    host_out, host_dst = out.cpu().numpy(), dst.cpu().numpy()
    ids, keep = pkg.shard.assign_identifiers(torch.from_numpy(draws.astype(np.int64)), base, layout, gfpc)
    for f in range(nf):  # one rank: global frame f is local frame f
        assert int(osz[f]) == int(sz[f])
        got = bytearray(host_out[int(offs[f]):int(offs[f]) + int(sz[f])])
        want = bytearray(host_dst[f * dstride:f * dstride + int(sz[f])])
        if not bool(keep[f]):
            want[8:14] = int(ids[f]).to_bytes(6, "big")
        assert got == want, f
    if layout != "streams" and secondary == 0:
        # a frame that made no draw (here: reported so) is refused, and nothing hangs
        bad = draws.copy()
        bad[1] = 0
        r = eng.gather(comm, 0, lay, gfpc, dst.data_ptr(), dstride, cap, sizes.data_ptr(), bad.ctypes.data, nf,
                       out.data_ptr(), out.numel(), offs.ctypes.data, osz.ctypes.data, base, pkg.GATHER_PATCH_IDS)
        assert api.error_name(r) == "PARAMS_INVALID"
        assert eng.synchronize() == 0
