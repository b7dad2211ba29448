#!/usr/bin/env python3
"""Checksum-enabled encode: a bench workload with
checksum_enabled=1, timed per call with HIP events (AIRS_CK_ALG=1|2 selects
the single-wave or the producer/consumer checksum kernel for comparison).  usage: ck_bench.py cfg2|cfg4"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = bench.load_pkg()
api = pkg.cmpapi
lib = pkg.load()
name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
wl = bench.WORKLOADS[name]
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
n, nf = wl["n"], wl["nctx"] * wl["fpc"]
stride = 2 * n
src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
for j, f in enumerate(bench.frame_ids(wl, 0, 1)):
    eng.synthesize(src.data_ptr() + j * stride, 2, wl["seed"], f, n, 1, stride, bench.noise_w(wl, f))
cap = lib.compress_bound(2 * n)
cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
dstride = (cap + 7) // 8 * 8
dst = torch.empty(nf * dstride, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
ctxs = pkg.context_array(1)
lib.initialise(ctxs[0], api.CmpParams(**dict(wl["params"], checksum_enabled=1)))
for k in range(2):
    assert eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for k in range(5):
    assert eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                        sizes.data_ptr()) == 0
e1.record(stream)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(json.dumps(dict(workload=name, checksum=True, alg=os.environ.get("AIRS_CK_ALG", "0"),
                      ms_per_call=round(ms, 4), GBps=round(nf * 2 * n / (ms * 1e-3) / 1e9, 1))))
