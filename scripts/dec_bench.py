#!/usr/bin/env python3
"""Decoder throughput: encode a bench workload on the
GPU, then time cmp_gpu_decompress of those frames (HIP events around the whole
call, host synchronisations of the parse included) and check the round trip.
Rate = decoded sample bytes / s.  usage: dec_bench.py cfg2|cfg4"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pkg = bench.load_pkg()
api = pkg.cmpapi
lib = pkg.load()
wname = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
wl = bench.WORKLOADS[wname]
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
n, nf = wl["n"], wl["frames"]
stride = 2 * n
src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
for j, f in enumerate(bench.frame_ids(wl, 0, 1)):
    eng.synthesize(src.data_ptr() + j * stride, 2, wl["seed"], f, n, 1, stride, wl["W"])
cap = lib.compress_bound(2 * n)
cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
cap = (cap + 7) // 8 * 8
dst = torch.empty(nf * cap, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
ctxs = pkg.context_array(1)
lib.initialise(ctxs[0], api.CmpParams(**bench.PARAMS))
assert eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), cap, cap,
                    sizes.data_ptr()) == 0
out = torch.empty(nf * n, dtype=torch.int16, device="cuda")
st = torch.zeros(nf, dtype=torch.int32, device="cuda")


def dec():
    assert eng.decompress(dst.data_ptr(), cap, cap, nf, out.data_ptr(), 2 * n, n, st.data_ptr()) == 0


for _ in range(2):
    dec()
torch.cuda.synchronize()
ms = []
for _ in range(5):
    t0 = time.perf_counter()
    dec()
    torch.cuda.synchronize()
    ms.append((time.perf_counter() - t0) * 1e3)
ms.sort()
ok = bool((st.cpu().numpy() == n).all()) and torch.equal(out.view(torch.uint8), src)
print(json.dumps(dict(workload=wname, frames=nf, samples_per_frame=n, decode_ms=round(ms[2], 4),
                      min_ms=round(ms[0], 4), GBps=round(nf * 2 * n / (ms[2] * 1e-3) / 1e9, 1),
                      roundtrip_ok=ok, note="wall clock of the whole call incl. host syncs")))
