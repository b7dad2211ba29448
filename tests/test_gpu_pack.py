"""cmp_gpu_pack_frames (the packing step of the multi-GPU gather, shard.py)
against shard.packed_offsets and host slicing: strided frames of random
sizes, error values in size slots, odd sizes, the frames cmp_gpu_compress
left in a batch buffer."""
import numpy as np
import pytest
import torch

from conftest import load_pkg

pytestmark = pytest.mark.gpu
pkg = load_pkg()
api = pkg.cmpapi


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine(torch.cuda.current_stream().cuda_stream)
    yield e
    e.close()


@pytest.mark.parametrize("nf,stride,cap", [(1, 64, 60), (7, 4104, 4100), (1024, 3048, 3000), (3000, 16, 16)])
def test_pack_frames_vs_slices(eng, nf, stride, cap):
    shard = pkg.shard
    rng = np.random.default_rng(nf)
    sizes = rng.integers(1, cap + 1, nf).astype(np.int64)
    sizes[rng.random(nf) < 0.1] = -30  # error values take no bytes
    src = torch.from_numpy(rng.integers(0, 256, nf * stride).astype(np.uint8)).cuda()
    sz = torch.from_numpy(sizes.astype(np.int32)).cuda()
    offs = shard.packed_offsets(torch.from_numpy(sizes))
    out = torch.full((int(offs[-1]) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    d_offs = torch.zeros(nf + 1, dtype=torch.int64, device="cuda")
    assert eng.pack_frames(src.data_ptr(), stride, cap, sz.data_ptr(), nf, out.data_ptr(), d_offs.data_ptr()) == 0
    assert eng.synchronize() == 0
    assert torch.equal(d_offs.cpu(), offs)
    h, o = src.cpu().numpy(), out.cpu().numpy()
    for j in range(nf):
        if sizes[j] > 0:
            a = int(offs[j])
            assert bytes(o[a:a + sizes[j]]) == bytes(h[j * stride:j * stride + sizes[j]]), j
    assert (o[int(offs[-1]):] == 0xEE).all()  # nothing past the packed total


def test_pack_frames_of_a_compress_batch(prod, eng):
    """shard.pack on the GPU (the gather's packing) of a real batch."""
    shard = pkg.shard
    n, nf = 5000, 40
    rng = np.random.default_rng(3)
    x = (np.cumsum(rng.integers(-30, 31, (nf, n)), axis=1) & 0xFFFF).astype(np.uint16)
    src = torch.from_numpy(x.reshape(-1).view(np.uint8).copy()).cuda()
    cap = prod.compress_bound(2 * n)
    dstride = (cap + 7) // 8 * 8
    dst = torch.zeros(nf * dstride, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = pkg.context_array(1)
    assert not api.is_error(prod.initialise(ctxs[0], api.CmpParams(primary_preprocessing=1, primary_encoder_type=1,
                                                                   primary_encoder_param=16)))
    assert eng.compress(ctxs, nf, "u16", src.data_ptr(), 2 * n, 2 * n, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0
    assert eng.synchronize() == 0
    offs = shard.packed_offsets(sizes.cpu())
    out = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    assert shard.pack(dst, dstride, sizes, nf, out, engine=eng, frame_capacity=cap) == int(offs[-1])
    torch.cuda.synchronize()
    ref = torch.empty_like(out.cpu())
    shard.pack(dst.cpu(), dstride, sizes.cpu(), nf, ref)
    assert torch.equal(out.cpu(), ref)
