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
if os.environ.get("AIRS_DBG"):  # ablation builds (-DAIRS_ABLATE=1) only: enc_common.h DBG() switches
    import ctypes
    lib.lib.airs_dev_set_debug.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
    lib.lib.airs_dev_set_debug(int(os.environ["AIRS_DBG"]), os.environ.get("AIRS_DBGTS_PATH", "").encode())
wl = dict(bench.WORKLOADS[sys.argv[1]])
if os.environ.get("AIRS_KB_FRAMES"):  # scaling probe: more frames of the same shape (no golden digest)
    wl["fpc"] = int(os.environ["AIRS_KB_FRAMES"])
stream = torch.cuda.current_stream()
eng = lib.engine(stream.cuda_stream)
if os.environ.get("AIRS_KB_EXCL"):  # the engine owns the device (CMP_GPU_OPT_EXCLUSIVE), as in bench.py
    assert eng.set_option(pkg.OPT_EXCLUSIVE, 1) == 0
n, nf = wl["n"], wl["nctx"] * wl["fpc"]
stride = 2 * n
# AIRS_KB_ROT=R: rotate over R input/output buffer sets (R >= 3 reads cold
# from HBM: the footprint exceeds the 256 MiB Infinity Cache); default 1 (warm)
ROT = int(os.environ.get("AIRS_KB_ROT", "1"))
srcs = [torch.empty(nf * stride, dtype=torch.uint8, device="cuda") for _ in range(ROT)]
for src in srcs:
    for j, f in enumerate(bench.frame_ids(wl, 0, 1)):
        eng.synthesize(src.data_ptr() + j * stride, 2, wl["seed"], f, n, 1, stride, bench.noise_w(wl, f))
cap = lib.compress_bound(2 * n)
cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
dstride = (cap + 7) // 8 * 8
dsts = [torch.empty(nf * dstride, dtype=torch.uint8, device="cuda") for _ in range(ROT)]
src, dst = srcs[0], dsts[0]
sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
ctxs = pkg.context_array(1)
lib.initialise(ctxs[0], api.CmpParams(**wl["params"]))
# AIRS_KB_AUTO=1: CMP_GPU_AUTO_RICE on any workload (no golden digest then)
flags = 1 if (wl.get("auto_rice") or os.environ.get("AIRS_KB_AUTO")) else 0
STREAM = bool(wl.get("stream"))  # cfg2s: one payload-only stream over every frame's samples
if STREAM:
    _p = wl["params"]

    class _StreamEng:
        """eng.compress's call shape over cmp_gpu_encode_stream (kbench only)"""

        def compress(self, ctxs_, nf_, kind, s, st, sb, d, dst_, cap_, sz, flags_=0):
            return eng.encode_stream(kind, s, nf_ * n, _p["primary_preprocessing"], _p["primary_encoder_type"],
                                     _p["primary_encoder_param"], 0, d, dst_ * nf_ - 64, sz)

        def synchronize(self):
            return eng.synchronize()
    eng_s = _StreamEng()
else:
    eng_s = eng
for k in range(10):
    assert eng_s.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                          sizes.data_ptr(), flags) == 0
# AIRS_KB_PRE=P: P more untimed launches over the rotated (cold) sets before
# the timed spans; AIRS_KB_IDLE=MS: then leave the GPU idle for MS ms
for k in range(int(os.environ.get("AIRS_KB_PRE", "0"))):
    assert eng_s.compress(ctxs, nf, "u16", srcs[k % ROT].data_ptr(), stride, stride, dsts[k % ROT].data_ptr(), dstride,
                        cap, sizes.data_ptr(), flags) == 0
torch.cuda.synchronize()
if os.environ.get("AIRS_KB_IDLE"):
    import time
    time.sleep(float(os.environ["AIRS_KB_IDLE"]) / 1e3)
ms = []
for rep in range(5):  # 5 spans of 20 back-to-back launches, one event pair each
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(20):
        src, dst = srcs[k % ROT], dsts[k % ROT]
        assert eng_s.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                              sizes.data_ptr(), flags) == 0
    e1.record(stream)
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1) / 20)
eng.synchronize()
ms.sort()
# bit-exactness of the last launch against the reference's golden digest
import hashlib  # noqa: E402
import numpy as np  # noqa: E402
sz = sizes.cpu().numpy().astype(np.uint32)
host = dst.cpu().numpy()
h = hashlib.sha256()
if STREAM:
    h.update(bytes(host[:int(sz[0])]))
    with open(os.path.join(bench.ROOT, "tests", "golden", "streams.json")) as f:
        want = json.load(f)["cases"][wl["golden"]]["sha256"]
else:
    for j in range(nf):
        b = bytearray(host[j * dstride:j * dstride + int(sz[j])])
        b[8:14] = b"\0" * 6
        h.update(b)
    with open(os.path.join(bench.ROOT, "tests", "golden", "configs.json")) as f:
        gold = json.load(f)["configs"][wl["golden"]]
    want = gold["shard_digests_n1"][0] if wl["layout"] == "roundrobin" else gold["digest"]
if os.environ.get("AIRS_KB_FRAMES") or (os.environ.get("AIRS_KB_AUTO") and not wl.get("auto_rice")):
    want = None
print(json.dumps(dict(workload=sys.argv[1], rot=ROT, dbg=os.environ.get("AIRS_DBG", "0"), median_ms=ms[len(ms) // 2],
                      min_ms=ms[0], GBps=round(nf * 2 * n / (ms[len(ms) // 2] * 1e-3) / 1e9, 1),
                      bitexact=(h.hexdigest() == want) if want else None, frames=nf)))
