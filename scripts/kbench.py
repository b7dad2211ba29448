#!/usr/bin/env python3
"""Kernel micro-benchmark: times cmp_gpu_compress on the bench workload with
HIP events; AIRS_DBG ablation modes are selected per process (env var), so
run this once per mode.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.argv += [] if len(sys.argv) > 1 else ["cfg2"]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = bench.load_pkg()
api = pkg.cmpapi
lib = pkg.load()
wl = bench.WORKLOADS[sys.argv[1]]
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
n, nf = wl["n"], wl["frames"]
stride = 2 * n
src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
for j, f in enumerate(bench.frame_ids(wl, 0, 1)):
    eng.synthesize(src.data_ptr() + j * stride, 2, wl["seed"], f, n, 1, stride, wl["W"])
cap = lib.compress_bound(2 * n)
cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
dstride = (cap + 7) // 8 * 8
dst = torch.empty(nf * dstride, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
ctxs = pkg.context_array(1)
lib.initialise(ctxs[0], api.CmpParams(**bench.PARAMS))
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
for k in range(40):
    if k >= 10:
        ev[k - 10][0].record(stream)
    assert eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0
    if k >= 10:
        ev[k - 10][1].record(stream)
torch.cuda.synchronize()
eng.synchronize()
ms = sorted(a.elapsed_time(b) for a, b in ev)
print(json.dumps(dict(workload=sys.argv[1], dbg=os.environ.get("AIRS_DBG", "0"), median_ms=ms[len(ms) // 2],
                      min_ms=ms[0], GBps=round(nf * 2 * n / (ms[len(ms) // 2] * 1e-3) / 1e9, 1))))
