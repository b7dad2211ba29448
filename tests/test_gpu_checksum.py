"""The device XXH32 frame checksum (reference lib/common/header.c:137-163:
XXH32, seed 419764627, over the samples as big-endian 16-bit words) of
checksum-enabled frames against the oracle: the producer/consumer kernel's
ring slots (256 stripes), partial slots, tails of 0-15 bytes, frames shorter
than one stripe, unaligned frame bases (the per-sample path), i16-in-i32
samples, and blocks of 16 frames with a partial last block."""
import numpy as np
import pytest
import torch

from conftest import load_pkg

pytestmark = pytest.mark.gpu
api = load_pkg().cmpapi


@pytest.fixture(scope="module")
def eng(prod):
    if not prod.gpu_available():
        pytest.fail("GPU test run without a usable HIP device")
    e = prod.engine(torch.cuda.current_stream().cuda_stream)
    yield e
    e.close()


@pytest.mark.parametrize("kind,n,nf,pad", [
    ("u16", 1, 3, 0), ("u16", 7, 5, 0), ("u16", 8, 17, 0), ("u16", 2048, 16, 0), ("u16", 2048 * 3 + 5, 33, 0),
    ("u16", 65536, 20, 0), ("u16", 1 << 20, 2, 0), ("u16", 5000, 9, 2), ("u16", 4099, 18, 6),
    ("i16_in_i32", 9, 4, 0), ("i16_in_i32", 2048 * 2 + 3, 17, 0), ("i16_in_i32", 70001, 5, 0),
    ("i16_in_i32", 3001, 6, 4)])
def test_checksum_vs_oracle(prod, eng, orc_ext, kind, n, nf, pad):
    rng = np.random.default_rng(n * 131 + nf)
    sb = 4 if kind == "i16_in_i32" else 2
    stride = n * sb + pad  # pad != 0: frame bases not 16-byte aligned
    stride += (-stride) % sb
    x = rng.integers(0, 1 << (8 * sb), (nf, stride // sb), dtype=np.uint64).astype(np.uint32 if sb == 4 else np.uint16)
    src = torch.from_numpy(x.reshape(-1).view(np.uint8).copy()).cuda()
    cap = 16 + 6 + 4 + 6 * n
    dstride = (cap + 7) // 8 * 8
    dst = torch.zeros(nf * dstride, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = (api.CmpContext * 1)()
    assert not api.is_error(prod.initialise(ctxs[0], api.CmpParams(primary_encoder_type=0, checksum_enabled=1)))
    assert eng.compress(ctxs, nf, kind, src.data_ptr(), stride, n * sb, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0
    assert eng.synchronize() == 0
    sz = sizes.cpu().numpy()
    out = dst.cpu().numpy()
    for f in range(nf):
        s = int(sz[f])
        assert s == 16 + 2 * n + 4, s
        got = int.from_bytes(bytes(out[f * dstride + s - 4:f * dstride + s]), "big")
        v = (x[f, :n] & 0xFFFF).astype(np.uint16)
        want = orc_ext.orc_checksum_u16(np.ascontiguousarray(v).ctypes.data, n)
        assert got == want, (f, hex(got), hex(want))
