#!/usr/bin/env python3
"""IWT encode throughput: NCTX contexts x 1 frame of N
u16 samples, primary IWT + GOLOMB_ZERO g=32, through one cmp_gpu_compress
call per step (the IWT coefficients go to each context's device work buffer,
then the encode kernel reads them as residuals).  Times STEPS launches with
one HIP event pair and checks FRAMES_CHECKED frames against the CPU oracle.
Prints one JSON line.  env: AIRS_IWT_N (65536), AIRS_IWT_CTX (1024)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = bench.load_pkg()
api = pkg.cmpapi
lib = pkg.load()
n = int(os.environ.get("AIRS_IWT_N", 65536))
nctx = int(os.environ.get("AIRS_IWT_CTX", 1024))
steps = 20
params = api.CmpParams(primary_preprocessing=2, primary_encoder_type=1, primary_encoder_param=32)
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
stride = 2 * n
src = torch.empty(nctx * stride, dtype=torch.uint8, device="cuda")
assert eng.synthesize(src.data_ptr(), 2, 0xA1A8, 0, n, nctx, stride, 32) == 0
cap = lib.compress_bound(2 * n)
dstride = (cap + 7) // 8 * 8
dst = torch.empty(nctx * dstride, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nctx, dtype=torch.int32, device="cuda")
wbs = lib.cal_work_buf_size(params, stride)
wstride = (wbs + 15) // 16 * 16
work = torch.zeros(nctx * wstride, dtype=torch.uint8, device="cuda")
ctxs = pkg.context_array(nctx)


def step():
    for c in range(nctx):  # a fresh primary pass each step (sequence number 0)
        assert not api.is_error(lib.initialise(ctxs[c], params, work.data_ptr() + c * wstride, wbs))
    assert eng.compress(ctxs, 1, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0


for _ in range(3):
    step()
torch.cuda.synchronize()
ms = []
for rep in range(3):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    tot = 0.0
    for k in range(steps):  # host-side context re-initialisation stays outside the timed span
        for c in range(nctx):
            lib.initialise(ctxs[c], params, work.data_ptr() + c * wstride, wbs)
        e0.record(stream)
        assert eng.compress(ctxs, 1, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                            sizes.data_ptr()) == 0
        e1.record(stream)
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1)
    ms.append(tot / steps)
eng.synchronize()
ms.sort()
# parity of a few frames against the CPU oracle (same params, fresh contexts)
orc = api.CmpLib(os.path.join(bench.ROOT, "oracle", "liborc.so"))
host = dst.cpu().numpy()
sz = sizes.cpu().numpy().astype(np.uint32)
xs = src.cpu().numpy()
ok = True
for f in (0, 1, nctx // 2, nctx - 1):
    x = xs[f * stride:(f + 1) * stride].view(np.uint16)
    c = api.CmpContext()
    wb = api.aligned_empty(wbs)
    orc.initialise(c, params, wb, wbs)
    d = api.aligned_empty(cap + 8)
    r = orc.compress_u16(c, d, cap, x)
    got = bytes(host[f * dstride:f * dstride + int(sz[f])])
    ref = bytes(d[:r]) if not api.is_error(r) else b""
    ok &= r == int(sz[f]) and ref[:8] == got[:8] and ref[14:] == got[14:]  # identifiers (bytes 8..13) differ
print(json.dumps(dict(workload=f"IWT + GOLOMB_ZERO g=32, {nctx} frames x {n} u16", median_ms=ms[1], min_ms=ms[0],
                      GBps=round(nctx * 2 * n / (ms[1] * 1e-3) / 1e9, 1), oracle_match=bool(ok))))
