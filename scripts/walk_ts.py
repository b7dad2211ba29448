#!/usr/bin/env python3
"""Walk-kernel timeline (ablation builds only: scripts/build_exp.sh NAME
"-DAIRS_ABLATE=1"): runs the cfg5 batch with AIRS_DBG bit 65536 and
summarises the per-(workgroup, acquisition) realtime stamps of enc_walk.hip
(wstamp: 0 samples ready, 1 after B1, 2 packed, 3 after B2, 4 after B3,
5 look-back done, 6 predecessor tail seen; 100 MHz clock).
usage: AIRS_LIB=exp/NAME/libairscmp.so python3 scripts/walk_ts.py OUT.json"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = sys.argv[1]
raw = out + ".bin"
pkg = bench.load_pkg()
lib = pkg.load()
lib.lib.airs_dev_set_debug.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
wl = dict(bench.WORKLOADS[os.environ.get("AIRS_WL", "cfg5")])
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
bs = bench.BufferSet(torch, pkg, lib, eng, wl, bench.frame_ids(wl, 0, 1))
for i in range(3):
    lib.lib.airs_dev_set_debug(65536 if i == 2 else 0, raw.encode())
    r = eng.compress(bs.ctxs, wl["fpc"], wl["kind"], bs.src.data_ptr(), bs.stride, bs.stride, bs.dst.data_ptr(),
                     bs.dstride, bs.cap, bs.sizes.data_ptr(), 0)
    assert r == 0, r
    assert eng.synchronize() == 0
fpc = wl["fpc"]
ts = np.fromfile(raw, dtype=np.uint64)
SEGN = int(os.environ.get("AIRS_TS_SEG", "4096"))  # samples per segment (2048: two data waves)
nb = wl["nctx"] * (wl["n"] // SEGN)
ts = ts[:nb * fpc * 8].reshape(nb, fpc, 8).astype(np.int64)
os.remove(raw)
t0 = ts[:, 0, 0].min()
us = lambda x: np.round(np.asarray(x, dtype=np.float64) * 0.01, 3)  # noqa: E731 (100 MHz ticks -> us)


def med(x):
    x = np.asarray(x)
    return float(us(np.median(x))) if x.size else None


def pct(x, q):
    x = np.asarray(x)
    return float(us(np.percentile(x, q))) if x.size else None


rel = ts[:, :, :7] - t0
start = rel[:, 0, 0]
end = rel[:, -1, 4]
spf = wl["n"] // SEGN
j = np.arange(nb) % spf
notfirst = j != 0
res = dict(
    kernel_span_us=float(us(end.max())),
    blocks=nb, fpc=fpc,
    block_start_us=dict(p0=pct(start, 0), p50=pct(start, 50), p90=pct(start, 90), p100=pct(start, 100)),
    block_life_us=dict(p10=pct(end - start, 10), p50=pct(end - start, 50), p90=pct(end - start, 90)),
    per_step_median_us=dict(
        phase1=med(rel[:, :, 1] - rel[:, :, 0]),
        pack=med(rel[:, :, 2] - rel[:, :, 1]),
        wait_B2=med(rel[:, :, 3] - rel[:, :, 2]),
        store=med(rel[:, :, 4] - rel[:, :, 3]),
        next_samples_ready=med(rel[:, 1:, 0] - rel[:, :-1, 4]),
        step_total=med(rel[:, 1:, 0] - rel[:, :-1, 0]),
        lb_after_B1=med((rel[:, :, 5] - rel[:, :, 1])[notfirst]),
        tail_after_lb=med((rel[:, :, 6] - rel[:, :, 5])[notfirst]),
        B2_after_tail=med((rel[:, :, 3] - rel[:, :, 6])[notfirst]),
    ),
    per_step_p90_us=dict(
        wait_B2=pct(rel[:, :, 3] - rel[:, :, 2], 90),
        lb_after_B1=pct((rel[:, :, 5] - rel[:, :, 1])[notfirst], 90),
        tail_after_lb=pct((rel[:, :, 6] - rel[:, :, 5])[notfirst], 90),
        step_total=pct(rel[:, 1:, 0] - rel[:, :-1, 0], 90),
    ),
    wait_B2_by_segment_us=[med((rel[:, :, 3] - rel[:, :, 2])[j == s]) for s in range(spf)],
    # where the slow workgroups are: lifetime (end - start) by segment index,
    # by stream, and by XCD (slot 7: HW_ID << 32 | XCC_ID)
    life_by_segment_us=[med((end - start)[j == s]) for s in range(spf)],
    life_by_stream_us=[med((end - start)[np.arange(nb) // spf == q]) for q in range(nb // spf)],
    end_by_stream_us=[float(us((end[np.arange(nb) // spf == q]).max())) for q in range(nb // spf)],
    life_by_xcd_us=[med((end - start)[(ts[:, 0, 7] & 0xF) == x]) for x in range(8)],
)
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
