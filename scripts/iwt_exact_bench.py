#!/usr/bin/env python3
"""IWT contexts with the uncompressed fallback (exact mode): NCTX contexts x
FPC acquisitions of N u16 samples, primary IWT, DIFF secondaries, the
fallback on, capacity = the raw frame size.  Times one cmp_gpu_compress call
(wall clock, to its synchronisation) in the device exact mode (round 5: IWT
passes run there) and host-stepped (CMP_GPU_HOST_STEPPED, the path IWT took
before).  Prints one JSON line.  env: AIRS_IWT_N (65536), AIRS_IWT_CTX (256),
AIRS_IWT_FPC (8)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = bench.load_pkg()
api = pkg.cmpapi
lib = pkg.load()
n = int(os.environ.get("AIRS_IWT_N", 65536))
nctx = int(os.environ.get("AIRS_IWT_CTX", 256))
fpc = int(os.environ.get("AIRS_IWT_FPC", 8))
params = api.CmpParams(primary_preprocessing=2, primary_encoder_type=1, primary_encoder_param=32,
                       secondary_iterations=3, secondary_preprocessing=1, secondary_encoder_type=1,
                       secondary_encoder_param=16, uncompressed_fallback_enabled=1)
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
stride = 2 * n
nf = nctx * fpc
src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
assert eng.synthesize(src.data_ptr(), 2, 0xA1A8, 0, n, nf, stride, 32) == 0
dstride = (lib.compress_bound(2 * n) + 7) // 8 * 8  # room for the worst case (asynchronous mode)
dst = torch.empty(nf * dstride, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
wbs = lib.cal_work_buf_size(params, stride)
wstride = (wbs + 15) // 16 * 16
work = torch.zeros(nctx * wstride, dtype=torch.uint8, device="cuda")
ctxs = pkg.context_array(nctx)


def run(flags):
    cap = 16 + 2 * n if params.uncompressed_fallback_enabled else lib.compress_bound(2 * n)
    for c in range(nctx):
        assert not api.is_error(lib.initialise(ctxs[c], params, work.data_ptr() + c * wstride, wbs))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eng.compress(ctxs, fpc, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, min(cap, dstride),
                     sizes.data_ptr(), flags)
    assert r == 0, api.error_name(r)
    assert eng.synchronize() == 0
    return (time.perf_counter() - t0) * 1e3


out = {"n": n, "contexts": nctx, "acquisitions": fpc}
for name, flags in (("device_exact", 0), ("host_stepped", api.GPU_HOST_STEPPED)):
    for _ in range(2):
        run(flags)
    ms = sorted(run(flags) for _ in range(7))
    out[name + "_ms"] = round(ms[len(ms) // 2], 3)
    out[name + "_sizes"] = int(sizes.sum().item())
out["speedup"] = round(out["host_stepped_ms"] / out["device_exact_ms"], 2)
# the asynchronous mode (no fallback, primary IWT passes only): one launch for
# the whole batch against one per acquisition step (CMP_GPU_STEPWISE)
params = api.CmpParams(primary_preprocessing=2, primary_encoder_type=1, primary_encoder_param=32)
for name, flags in (("async_one_launch", 0), ("async_stepwise", api.GPU_STEPWISE)):
    for _ in range(2):
        run(flags)
    ms = sorted(run(flags) for _ in range(7))
    out[name + "_ms"] = round(ms[len(ms) // 2], 3)
    out[name + "_sizes"] = int(sizes.sum().item())
out["input_GBps_device_exact"] = round(nf * stride / out["device_exact_ms"] / 1e6, 1)
print(json.dumps(out))
