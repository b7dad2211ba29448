#!/usr/bin/env python3
"""Where does the bench step's wall time go?  (a) host time per
cmp_gpu_compress call (no sync), (b) wall per step with and without per-step
HIP events, (c) kernel time from events."""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
pkg = bench.load_pkg(); api = pkg.cmpapi; lib = pkg.load()
wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "cfg2"]
stream = torch.cuda.current_stream(); eng = lib.engine(stream.cuda_stream)
n, nf = wl["n"], wl["frames"]; stride = 2 * n
src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
eng.synthesize(src.data_ptr(), 2, wl["seed"], 0, n, nf, stride, wl["W"])
cap = lib.compress_bound(2 * n); cap = cap if not api.is_error(cap) else 3 * 2 * n + 64; dstride = (cap + 7) // 8 * 8
dst = torch.empty(nf * dstride, dtype=torch.uint8, device="cuda")
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
ctxs = pkg.context_array(1); lib.initialise(ctxs[0], api.CmpParams(**bench.PARAMS))
def step():
    r = eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap, sizes.data_ptr())
    assert r == 0, api.error_name(r)
for _ in range(10): step()
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for _ in range(K): step()
t1 = time.perf_counter()
torch.cuda.synchronize(); t2 = time.perf_counter()
host_us = (t1 - t0) / K * 1e6; wall_noev = (t2 - t0) / K * 1e6
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
torch.cuda.synchronize(); t0 = time.perf_counter()
for a, b in ev:
    a.record(stream); step(); b.record(stream)
torch.cuda.synchronize(); t2 = time.perf_counter()
wall_ev = (t2 - t0) / K * 1e6
kern = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)[K // 2]
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); e0.record(stream)
for _ in range(K): step()
e1.record(stream); torch.cuda.synchronize()
gpu_span = e0.elapsed_time(e1) * 1e3 / K
print(json.dumps(dict(host_call_us=round(host_us, 2), wall_per_step_no_events_us=round(wall_noev, 2),
                      wall_per_step_events_us=round(wall_ev, 2), kernel_us_events=round(kern, 2),
                      gpu_span_per_step_us=round(gpu_span, 2))))
