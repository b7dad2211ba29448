#!/usr/bin/env python3
"""bench.py -- AIRSPACE encode throughput on MI355X.

One step = one cmp_gpu_compress() call over this rank's batch of frames whose
samples are already resident in HBM (BASELINE.json metric: encode GB/s on the
uncompressed input, 1 GB = 1e9 B, bit-exact vs the CPU reference).

Workloads (BASELINE.json configs):

  cfg2  (default at N = 1) configs[1]: 64 Mi u16 samples as 16 frames x 4 Mi
        (the 24-bit header size field caps a frame at 8 388 607 samples),
        DIFF + GOLOMB_ZERO g = 32
  cfg3  configs[2]: 1024 frames x 64 Ki u16, W_f = 2^(f mod 12), DIFF +
        GOLOMB_ZERO with the per-frame Rice k (CMP_GPU_AUTO_RICE)
  cfg4  (default at N > 1) configs[3]: frames of 64 Ki u16 sharded round-robin,
        1024 per rank (weak scaling: 128 MiB per GPU, N = 8 is the 8192-frame
        config); the compressed frames are then gathered to rank 0 (timed
        separately, not part of `value`)
  cfg5  configs[4]: 256 streams x 16 acquisitions x 64 Ki i16-in-i32 samples;
        acquisition 0 DIFF + ZERO g = 16, 1-15 MODEL + MULTI g = 8 o = 107
        rate 11 (one step = all 4096 frames, 16 launches)

Cold inputs: the timed steps rotate over enough input/output buffer sets that
one rotation touches more than the 256 MiB Infinity Cache, so every step reads
its samples from HBM (MI355X_MICROARCH.md, Infinity Cache residency rule).  A
warm replay of one buffer set is reported beside it under "warm".

Prints ONE JSON line on rank 0.  Diagnostics go to stderr.
"""
import argparse
import ctypes
import hashlib
import importlib.util
import json
import math
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "airs-compression_amd")
METRIC = "encode GB/s (uncompressed in) on 16-bit frames; bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
INFINITY_CACHE = 256 << 20
DIFF, MODEL, ZERO, MULTI = 1, 3, 1, 2


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "airs_compression_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["airs_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


CFG_ZERO32 = dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO, primary_encoder_param=32)
WORKLOADS = {
    "cfg2": dict(desc="configs[1]: 64 Mi u16 samples as 16 frames x 4 Mi, DIFF + GOLOMB_ZERO g=32",
                 kind="u16", n=4 << 20, nctx=1, fpc=16, seed=0xA1A6, W=32, golden="cfg2_64Mi",
                 layout="block", params=CFG_ZERO32),
    "cfg2s": dict(desc="configs[1] literally: ONE 64 Mi-sample u16 stream, payload only (no header, no 24-bit "
                       "frame limit: cmp_gpu_encode_stream), DIFF + GOLOMB_ZERO g=32; the cfg2 samples",
                  kind="u16", n=4 << 20, nctx=1, fpc=16, seed=0xA1A6, W=32, golden="cfg2_stream",
                  layout="block", stream=True, params=CFG_ZERO32),
    "cfg3": dict(desc="configs[2]: 1024 frames x 64 Ki u16, W_f = 2^(f mod 12), DIFF + GOLOMB_ZERO with "
                      "the per-frame Rice k (CMP_GPU_AUTO_RICE)",
                 kind="u16", n=64 << 10, nctx=1, fpc=1024, seed=0xA1A7, W="pow2_mod12", golden="cfg3_autorice",
                 layout="block", auto_rice=True, params=CFG_ZERO32),
    "cfg4": dict(desc="configs[3]: frames of 64 Ki u16, round-robin over GPUs (1024 per GPU), "
                      "DIFF + GOLOMB_ZERO g=32",
                 kind="u16", n=64 << 10, nctx=1, fpc=1024, seed=0xA1A8, W=32, golden="cfg4_8192",
                 layout="roundrobin", params=CFG_ZERO32),
    "cfg5": dict(desc="configs[4]: 256 streams x 16 acquisitions x 64 Ki i16-in-i32 samples (256 Mi), "
                      "primary DIFF + GOLOMB_ZERO g=16, secondary MODEL + GOLOMB_MULTI g=8 o=107 rate=11",
                 kind="i16_in_i32", n=64 << 10, nctx=256, fpc=16, seed=0xA1A9, W=32, golden="cfg5_model",
                 layout="streams",
                 params=dict(primary_preprocessing=DIFF, primary_encoder_type=ZERO, primary_encoder_param=16,
                             secondary_iterations=15, secondary_preprocessing=MODEL,
                             secondary_encoder_type=MULTI, secondary_encoder_param=8,
                             secondary_encoder_outlier=107, model_rate=11)),
}
# configs[4] as ONE GPU of an 8-GPU node holds it (streams s mod 8, rank 0's
# shard: 32 streams): the per-GPU work of the 8-GPU strong-scaling run of
# configs[4]
WORKLOADS["cfg5s8"] = dict(WORKLOADS["cfg5"], nctx=32, shard=(0, 8),
                           desc="configs[4], rank 0's shard at N = 8: streams 0, 8, ..., 248 (32 streams x 16 "
                                "acquisitions x 64 Ki i16-in-i32), parameters of cfg5")
# configs[4] with the uncompressed fallback enabled: every frame may fall back,
# so the batch runs the context state machine on the device (the frames are
# those of cfg5: this data always compresses)
WORKLOADS["cfg5fb"] = dict(WORKLOADS["cfg5"], desc=WORKLOADS["cfg5"]["desc"] + ", uncompressed fallback enabled",
                           params=dict(WORKLOADS["cfg5"]["params"], uncompressed_fallback_enabled=1))
# rank 0's shard at N = 8 with the fallback enabled: 32 contexts are too few for
# the context walk, so the batch takes the speculative segment walk (one launch,
# then one read-back of the statuses; contexts with a frame that does not fit
# run again on the device state machine: none here)
WORKLOADS["cfg5fbs8"] = dict(WORKLOADS["cfg5s8"], desc=WORKLOADS["cfg5s8"]["desc"] + ", uncompressed fallback enabled",
                             params=dict(WORKLOADS["cfg5"]["params"], uncompressed_fallback_enabled=1))


def sample_bytes(wl):
    return 4 if wl["kind"] == "i16_in_i32" else 2


def noise_w(wl, f):
    return (1 << (f % 12)) if wl["W"] == "pow2_mod12" else wl["W"]


def algorithmic_bytes(wl):
    """Compulsory HBM reads of one step: the samples (2 B,
    or 4 B for i16-in-i32), plus the 2 B model read of every MODEL pass."""
    n, nf = wl["n"], wl["nctx"] * wl["fpc"]
    b = nf * n * sample_bytes(wl)
    if wl["params"].get("secondary_preprocessing") == MODEL:
        sec = wl["nctx"] * min(wl["fpc"] - 1, wl["params"]["secondary_iterations"])
        b += sec * n * 2
    return b


def measured_traffic(wname):
    """HBM bytes per step of the encode path from the latest committed PMC
    passes (profiles/rNN_traffic_<workload>.json, written by scripts/traffic.py
    from rocprofv3 FETCH_SIZE / WRITE_SIZE runs of this bench command), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{wname}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f)
    return t.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def frame_ids(wl, rank, world):
    """global frame numbers of this rank's frames, in local order (shard.py layouts)"""
    nf, fpc = wl["nctx"] * wl["fpc"], wl["fpc"]
    if wl.get("shard"):  # one fixed rank's shard of a larger node (cfg5s8)
        rank, world = wl["shard"]
    if wl["layout"] == "roundrobin":
        return [rank + world * j for j in range(nf)]
    if wl["layout"] == "streams":  # stream s on rank s mod N (its model stays on one GPU)
        return [(rank + world * i) * fpc + a for i in range(wl["nctx"]) for a in range(fpc)]
    return [rank * nf + j for j in range(nf)]


def host_cpu_info():
    """CPU resources this job may use: logical CPUs, affinity and the cgroup
    CPU quota (the GPU box grants a share of a large host)."""
    info = dict(logical_cpus=os.cpu_count(), affinity=len(os.sched_getaffinity(0)))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            info["cgroup_cpu_quota"] = round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    info["nproc"] = subprocess.run(["nproc"], capture_output=True, text=True).stdout.strip()
    usable = info["affinity"]
    if "cgroup_cpu_quota" in info:
        usable = min(usable, max(1, int(info["cgroup_cpu_quota"])))
    info["usable_cpus"] = usable
    return info


def cpu_baseline(wl):
    """The reference's own CPU path (oracle/_ref/libref.so, compiled from the
    reference sources) timed on this host over every CPU this job may use:
    OpenMP over streams, one context per thread.  Falls back to the clean-room
    port (oracle/liborc.so) where the reference was not built."""
    api = sys.modules["airs_compression_amd"].cmpapi
    ref = os.path.join(ROOT, "oracle", "_ref", "libref.so")
    orc = os.path.join(ROOT, "oracle", "liborc.so")
    path, kind = (ref, "reference") if os.path.exists(ref) else (orc, "port")
    cpu = host_cpu_info()
    if wl.get("stream"):
        return cpu_baseline_stream(wl, path, kind, orc, cpu)
    threads = cpu["usable_cpus"]
    gen = ctypes.CDLL(orc, mode=ctypes.RTLD_LOCAL)
    gen.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    gen.orc_synth_i32.argtypes = gen.orc_synth_u16.argtypes
    n, sb = wl["n"], sample_bytes(wl)
    # bounded sample: every frame of cfg2/cfg3/cfg4, 64 of cfg5's 256 streams
    nctx = min(wl["nctx"], 64)
    fpc = wl["fpc"]
    nf = nctx * fpc
    # one context owning all frames (cfg2, cfg4) is a serial chain in the
    # reference; its frames are independent data, so the CPU baseline gives
    # every frame its own context and runs them on all usable CPUs (the
    # primary passes are identical; identifiers and sequence numbers differ)
    split = nctx == 1 and fpc > 1 and not wl["params"].get("secondary_iterations")
    if split:
        nctx, fpc = nf, 1
    data = np.empty((nf, n), dtype=np.int32 if sb == 4 else np.uint16)
    for j, f in enumerate(frame_ids(wl, 0, 1)[:nf]):
        (gen.orc_synth_i32 if sb == 4 else gen.orc_synth_u16)(wl["seed"], f, n, noise_w(wl, f), data[j].ctypes.data)
    drv = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    drv.drv_run.restype = ctypes.c_uint64
    drv.drv_run_autorice.restype = ctypes.c_uint64
    lib = api.CmpLib(path)
    cap = lib.compress_bound(2 * n)
    cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
    stride = (cap + 7) // 8 * 8
    dst = api.aligned_empty(stride * nf)
    sizes = np.zeros(nf, dtype=np.uint32)
    prm = api.CmpParams(**wl["params"])
    k_of = {"u16": 0, "i16": 1, "i16_in_i32": 2}[wl["kind"]]

    def run(th):
        t0 = time.perf_counter()
        if wl.get("auto_rice"):
            tot = drv.drv_run_autorice(ctypes.byref(prm), k_of, ctypes.c_void_p(data.ctypes.data),
                                       ctypes.c_uint32(sb * n), ctypes.c_uint64(sb * n), ctypes.c_uint32(nf),
                                       ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                                       ctypes.c_void_p(sizes.ctypes.data), None, ctypes.c_int(th), ctypes.c_int(1))
        else:
            tot = drv.drv_run(ctypes.byref(prm), k_of, ctypes.c_void_p(data.ctypes.data), ctypes.c_uint32(sb * n),
                              ctypes.c_uint64(sb * n), ctypes.c_uint32(nctx), ctypes.c_uint32(fpc),
                              ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                              ctypes.c_void_p(sizes.ctypes.data), ctypes.c_int(th), ctypes.c_int(1))
        dt = time.perf_counter() - t0
        assert tot != 2**64 - 1
        return dt

    run(threads)  # warm-up
    times = sorted(run(threads) for _ in range(5))
    best = times[0]
    nbytes = nf * sb * n
    single_nf = max(1, nf // 16)  # single-thread leg on a slice (bounded time)
    out = dict(value=round(nbytes / best / 1e9, 4), unit="GB/s", cores=threads, kind=kind,
               sample=f"{nf} frames x {n} samples ({nbytes / 2**20:.0f} MiB of {wl['kind']} input, the same "
                      f"synthetic frames and parameters as the GPU workload), best of 5 after a warm-up, "
                      f"OpenMP over {'frames' if wl.get('auto_rice') or split else 'streams'}, one context per "
                      f"{'frame' if split else 'thread'}",
               median_value=round(nbytes / times[2] / 1e9, 4), host=cpu,
               cores_note=(f"{threads} threads = every CPU this job may use: the GPU box's cgroup grants "
                           f"{cpu.get('cgroup_cpu_quota', 'no')} CPUs of the host's {cpu['logical_cpus']} "
                           f"logical CPUs"))
    # single thread on the first 1/16 of the frames
    if not wl.get("auto_rice"):
        nctx1 = max(1, nctx // 16) if nctx > 1 else 1
        fpc1 = fpc if nctx > 1 else max(1, fpc // 16)
        t0 = time.perf_counter()
        tot = drv.drv_run(ctypes.byref(prm), k_of, ctypes.c_void_p(data.ctypes.data), ctypes.c_uint32(sb * n),
                          ctypes.c_uint64(sb * n), ctypes.c_uint32(nctx1), ctypes.c_uint32(fpc1),
                          ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                          ctypes.c_void_p(sizes.ctypes.data), ctypes.c_int(1), ctypes.c_int(1))
        dt = time.perf_counter() - t0
        assert tot != 2**64 - 1
        single_nf = nctx1 * fpc1
    else:
        t0 = time.perf_counter()
        tot = drv.drv_run_autorice(ctypes.byref(prm), k_of, ctypes.c_void_p(data.ctypes.data),
                                   ctypes.c_uint32(sb * n), ctypes.c_uint64(sb * n), ctypes.c_uint32(single_nf),
                                   ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                                   ctypes.c_void_p(sizes.ctypes.data), None, ctypes.c_int(1), ctypes.c_int(1))
        dt = time.perf_counter() - t0
        assert tot != 2**64 - 1
    out["single_thread_value"] = round(single_nf * sb * n / dt / 1e9, 4)
    return out


def cpu_baseline_stream(wl, path, kind, orc, cpu):
    """One payload-only stream is one serial encoder loop on the CPU (the
    reference's internal encoder API, oracle/ref_payload.c): one thread, on
    the first 4 of the 16 frames' samples (16 Mi samples)."""
    gen = ctypes.CDLL(orc, mode=ctypes.RTLD_LOCAL)
    gen.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    fn = lib.ref_payload_stream if kind == "reference" else lib.orc_payload_stream
    fn.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p, ctypes.c_uint32]
    fn.restype = ctypes.c_uint32
    n, frames = wl["n"], 4
    x = np.empty(frames * n, dtype=np.uint16)
    for f in range(frames):
        gen.orc_synth_u16(wl["seed"], f, n, wl["W"], x[f * n:].ctypes.data)
    cap = 3 * frames * n + 64
    dst = np.zeros(cap + 8, dtype=np.uint8)
    off = (-dst.ctypes.data) % 8
    p = wl["params"]
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        r = fn(x.ctypes.data, frames * n, 0, p["primary_preprocessing"], p["primary_encoder_type"],
               p["primary_encoder_param"], 0, dst.ctypes.data + off, cap)
        times.append(time.perf_counter() - t0)
        assert r < 0xFFFFFF00
    nbytes = x.nbytes
    return dict(value=round(nbytes / min(times) / 1e9, 4), unit="GB/s", cores=1, kind=kind,
                sample=f"one stream of {frames * n} u16 samples ({nbytes / 2**20:.0f} MiB, the first 4 of the 16 "
                       f"cfg2 frames), best of 3, {'oracle/ref_payload.c over the reference encoder' if kind == 'reference' else 'orc_payload_stream'}",
                host=cpu, cores_note="a single stream is one serial bit-writer loop: one thread")


class BufferSet:
    """Device buffers of one copy of the workload: inputs, outputs, sizes,
    contexts (and their device work buffers)."""

    def __init__(self, torch, pkg, lib, eng, wl, fids):
        api = pkg.cmpapi
        n, sb = wl["n"], sample_bytes(wl)
        self.nctx, self.fpc = wl["nctx"], wl["fpc"]
        nf = self.nctx * self.fpc
        self.stride = n * sb
        self.src = torch.empty(nf * self.stride, dtype=torch.uint8, device="cuda")
        if wl["W"] == "pow2_mod12" or fids != list(range(fids[0], fids[0] + nf)):
            for j, f in enumerate(fids):
                assert eng.synthesize(self.src.data_ptr() + j * self.stride, sb, wl["seed"], f, n, 1, self.stride,
                                      noise_w(wl, f)) == 0
        else:
            assert eng.synthesize(self.src.data_ptr(), sb, wl["seed"], fids[0], n, nf, self.stride, wl["W"]) == 0
        cap = lib.compress_bound(2 * n)
        self.cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
        self.dstride = (self.cap + 7) // 8 * 8
        self.dst = torch.empty(nf * self.dstride, dtype=torch.uint8, device="cuda")
        self.sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
        prm = api.CmpParams(**wl["params"])
        wbs = lib.cal_work_buf_size(prm, self.stride)
        wstride = (wbs + 15) // 16 * 16
        self.work = torch.zeros(max(self.nctx * wstride, 16), dtype=torch.uint8, device="cuda")
        self.ctxs = pkg.context_array(self.nctx)
        for c in range(self.nctx):
            r = lib.initialise(self.ctxs[c], prm, (self.work.data_ptr() + c * wstride) if wbs else None, wbs)
            assert not api.is_error(r), api.error_name(r)
        self.nbytes = self.src.numel() + self.dst.numel() + self.work.numel()


def make_step(api, eng, wl, draws):
    """One step: one cmp_gpu_compress call over a buffer set (or one payload-only
    stream for cfg2s)."""
    fpc = wl["fpc"]
    flags = 1 if wl.get("auto_rice") else 0
    nf = wl["nctx"] * fpc

    def step(bs):
        if wl.get("stream"):  # one payload-only stream over all the samples of the set
            p = wl["params"]
            r = eng.encode_stream(wl["kind"], bs.src.data_ptr(), nf * wl["n"], p["primary_preprocessing"],
                                  p["primary_encoder_type"], p["primary_encoder_param"], 0, bs.dst.data_ptr(),
                                  bs.dst.numel() - 64, bs.sizes.data_ptr())
            if r:
                raise RuntimeError("cmp_gpu_encode_stream: " + api.error_name(r))
            return
        r = eng.compress(bs.ctxs, fpc, wl["kind"], bs.src.data_ptr(), bs.stride, bs.stride, bs.dst.data_ptr(),
                         bs.dstride, bs.cap, bs.sizes.data_ptr(), flags, draws.ctypes.data)
        if r:
            raise RuntimeError("cmp_gpu_compress: " + api.error_name(r))
    return step


def timed_steps(torch, stream, step, bsets, steps, warmup, sync):
    """W untimed steps, then K timed ones bracketed by sync() and a device
    synchronisation on both sides: (wall seconds, HIP-event ms per step)."""
    for i in range(warmup):
        step(bsets[i % len(bsets)])
    torch.cuda.synchronize()
    # one HIP event pair around the K steps (on the engine's stream): a
    # pair per step would itself add ~8 us of stream time per step
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        step(bsets[i % len(bsets)])
    ev1.record(stream)
    torch.cuda.synchronize()
    sync()
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_time(ev1) / steps


def per_launch_us(torch, stream, step, bsets, n):
    """The per-launch spread of the same cold steps (the mean of
    the timed region hides a bimodal kernel): n more steps over the rotated
    sets, each between its own HIP event pair on the engine stream.  Not
    part of `value` (an event pair per step adds stream time of its own)."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    torch.cuda.synchronize()
    for i, (e0, e1) in enumerate(evs):
        e0.record(stream)
        step(bsets[i % len(bsets)])
        e1.record(stream)
    torch.cuda.synchronize()
    us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in evs)
    return dict(n=n, min=round(us[0], 2), p50=round(us[n // 2], 2), p90=round(us[(9 * n) // 10], 2),
                max=round(us[-1], 2), max_over_min=round(us[-1] / us[0], 3),
                note="each step of a separate cold pass after the timed region between its own HIP events "
                     "(diagnostic: the spread of single launches, not part of value)")


def make_sets(torch, pkg, lib, eng, wl, fids, rotate):
    """The buffer sets the timed steps rotate over: enough that one rotation
    touches more than the Infinity Cache (cold reads)."""
    sets = [BufferSet(torch, pkg, lib, eng, wl, fids)]
    rot = rotate or max(1, math.ceil(1.25 * INFINITY_CACHE / sets[0].nbytes))
    rot = max(rot, 3) if sets[0].src.numel() < INFINITY_CACHE else rot
    for _ in range(rot - 1):
        sets.append(BufferSet(torch, pkg, lib, eng, wl, fids))
    torch.cuda.synchronize()
    return sets


def scaling_reference_n1(torch, pkg, lib, eng, stream, steps, warmup):
    """cfg4 on this one GPU (rank 0's 1024 frames at N = 1): the per-GPU work of
    every N > 1 run, so that their value / (N x this) is the scaling
    efficiency against the same workload (the N = 1 line itself is cfg2)."""
    wl = WORKLOADS["cfg4"]
    nf = wl["nctx"] * wl["fpc"]
    draws = np.zeros(nf, dtype=np.uint8)
    sets = make_sets(torch, pkg, lib, eng, wl, frame_ids(wl, 0, 1), 0)
    wall, kern = timed_steps(torch, stream, make_step(pkg.cmpapi, eng, wl, draws), sets, steps, warmup, lambda: None)
    del sets
    torch.cuda.empty_cache()
    return dict(workload="cfg4", n_gpus=1, frames=nf,
                value=round(nf * 2 * wl["n"] * steps / wall / 1e9, 3), unit="GB/s",
                ms_per_step=round(wall / steps * 1e3, 5), avg_step_gpu_ms=round(kern, 5),
                note="the per-GPU workload of the N > 1 lines (cfg4: 1024 frames per GPU) on one GPU; "
                     "weak-scaling efficiency at N = value_N / (N x this value)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None)
    ap.add_argument("--rotate", type=int, default=0,
                    help="buffer sets to rotate over (0: enough to exceed the 256 MiB Infinity Cache)")
    ap.add_argument("--no-warm", action="store_true", help="skip the warm (one buffer set) replay")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--scaling-reference", action="store_true",
                    help="with --workload at N = 1: also time cfg4 (the per-GPU work of the N > 1 runs)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # AIRS_BENCH_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # fewer GPUs (use with --no-gather); the measured runs use RCCL ("nccl")
    backend = os.environ.get("AIRS_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev else local
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    pkg = load_pkg()
    api = pkg.cmpapi
    lib = pkg.load()
    assert lib.gpu_available(), "no HIP device"
    stream = torch.cuda.current_stream()
    eng = lib.engine(stream.cuda_stream)
    # this process owns its GPU for the run (one rank per GPU, nothing else on
    # the device while the timed kernels run): the MODEL segment walk may order
    # its workgroups by block index (include/cmp_gpu.h CMP_GPU_OPT_EXCLUSIVE)
    assert eng.set_option(pkg.OPT_EXCLUSIVE, 1) == 0

    wname = args.workload or ("cfg2" if world == 1 else "cfg4")
    wl = WORKLOADS[wname]
    if world > 1 and wl["layout"] not in ("roundrobin", "streams"):
        raise SystemExit(f"--workload {wname} is a single-GPU config; N > 1 runs cfg4 (round-robin frames) or "
                         f"cfg5 (streams)")
    n, nctx, fpc = wl["n"], wl["nctx"], wl["fpc"]
    nf = nctx * fpc
    sb = sample_bytes(wl)
    fids = frame_ids(wl, rank, world)

    sets = make_sets(torch, pkg, lib, eng, wl, fids, args.rotate)

    draws = np.zeros(nf, dtype=np.uint8)  # identifier draws per frame (cmp_gpu_batch.draws), for the gather
    step = make_step(api, eng, wl, draws)

    def timed(bsets, steps, warmup, sync=barrier):
        return timed_steps(torch, stream, step, bsets, steps, warmup, sync)

    wall, kern_avg_ms = timed(sets, args.steps, args.warmup)
    t = torch.tensor([wall], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    launch_us = None
    if world == 1:
        launch_us = per_launch_us(torch, stream, step, sets, 20)
    warm = None
    if not args.no_warm and world == 1:
        wwall, wkern = timed(sets[:1], args.steps, 2)
        warm = dict(value=round(nf * sb * n * args.steps / wwall / 1e9, 3), ms_per_step=round(wwall / args.steps * 1e3, 5),
                    avg_step_gpu_ms=round(wkern, 5),
                    note="same K steps replayed on ONE buffer set (inputs may be served by the Infinity Cache)")

    # ---- the single-GPU reference of the scaling runs (not in `value`) -----
    scaling_ref = None
    if world == 1 and wname != "cfg4" and (args.workload is None or args.scaling_reference):
        scaling_ref = scaling_reference_n1(torch, pkg, lib, eng, stream, args.steps, args.warmup)
    elif world > 1:
        # rank 0 replays its own shard alone (the other ranks wait): the same
        # per-GPU work with nothing else on the node
        barrier()
        if rank == 0:
            swall, skern = timed(sets, args.steps, 2, sync=lambda: None)
            scaling_ref = dict(workload=wname, n_gpus=1, frames=nf,
                               value=round(nf * sb * n * args.steps / swall / 1e9, 3), unit="GB/s",
                               ms_per_step=round(swall / args.steps * 1e3, 5), avg_step_gpu_ms=round(skern, 5),
                               note="rank 0's shard replayed on its GPU alone after the timed run (other ranks "
                                    "idle): the one-GPU rate of the per-GPU work")
        barrier()

    # ---- bit-exactness against the reference's golden digests (every set) --
    gfile = "streams.json" if wl.get("stream") else "configs.json"
    with open(os.path.join(ROOT, "tests", "golden", gfile)) as f:
        gold = json.load(f)["cases" if wl.get("stream") else "configs"][wl["golden"]]
    key = f"shard_digests_n{world}" if wl["layout"] == "roundrobin" else None
    if wl.get("shard"):
        want = gold[f"shard_digests_n{wl['shard'][1]}"][wl["shard"][0]] if world == 1 else None
    elif key and key in gold:
        want = gold[key][rank]
    elif wl["layout"] in ("block", "streams") and world == 1:
        want = gold["sha256"] if wl.get("stream") else gold["digest"]
    else:
        want = None
    bitexact = None
    comp_bytes = 0
    for bs in sets:
        if wl.get("stream"):
            sz0 = int(bs.sizes[:1].cpu().numpy().astype(np.uint32)[0])
            if api.is_error(sz0):
                raise RuntimeError("stream error " + api.error_name(sz0))
            h = hashlib.sha256(bytes(bs.dst[:sz0].cpu().numpy())).hexdigest()
            ok = h == gold["sha256"]
            bitexact = ok if bitexact is None else (bitexact and ok)
            comp_bytes = sz0
            continue
        sz = bs.sizes.cpu().numpy().astype(np.uint32)
        errs = [api.error_name(int(s)) for s in sz if api.is_error(int(s))]
        if errs:
            raise RuntimeError(f"frame errors: {errs[:4]}")
        host = bs.dst.cpu().numpy()
        h = hashlib.sha256()
        for j in range(nf):
            b = bytearray(host[j * bs.dstride:j * bs.dstride + int(sz[j])])
            b[8:14] = b"\0" * 6
            h.update(b)
        ok = (h.hexdigest() == want) if want else None
        bitexact = ok if bitexact is None else (bitexact and ok)
        comp_bytes = int(sz.astype(np.uint64).sum())
        del host

    # ---- gather of compressed frames to rank 0 (not in `value`) -----------
    gather = None
    if world > 1 and not args.no_gather:
        bs = sets[0]
        # identifiers of one process over the node's frames with the default
        # counter (first draw 0): one context per stream, initialised in
        # stream order, so the frame draws start after nctx_total - 1
        nstreams = world * nctx if wl["layout"] == "streams" else 1
        gather, g = pkg.shard.gather_frames_timed(dist, bs.dst, bs.dstride, bs.sizes, nf, rank, world,
                                                  layout=wl["layout"], patch_base=nstreams - 1, engine=eng,
                                                  frame_capacity=bs.cap, draws=draws, fpc=fpc)
        if g is not None:
            host_all = g.data.cpu().numpy()
            offs, lens = g.offsets.cpu().numpy(), g.sizes.numpy()
            hg = hashlib.sha256()
            for f in range(g.num_frames):
                b = bytearray(host_all[offs[f]:offs[f] + lens[f]])
                # cfg4: one draw per frame; cfg5: one per stream (its primary frame)
                want_id = 1 + f if wl["layout"] != "streams" else nstreams + f // fpc
                ok_id = int.from_bytes(b[8:14], "big") == want_id
                b[8:14] = b"\0" * 6
                hg.update(b)
                if not ok_id:
                    gather["identifier_patch_ok"] = False
            gather.setdefault("identifier_patch_ok", True)
            gwant = gold.get(f"gather_digest_n{world}")
            gather["bitexact_vs_reference"] = (hg.hexdigest() == gwant) if gwant else None
            del g, host_all

    in_bytes_rank = nf * sb * n
    alg_bytes = algorithmic_bytes(wl)
    total_in = in_bytes_rank * world
    value = total_in * args.steps / wall_max / 1e9
    ms_step = wall_max / args.steps * 1e3
    traffic, traffic_src = measured_traffic(wname)
    achieved = alg_bytes / (kern_avg_ms * 1e-3) / 1e9
    rice = ("airs::rice_kernel<DIFF> (enc_rice.hip: 16 Ki-sample segments, codeword pairs from phase 1, one LDS "
            "arena per segment, decoupled look-back)")
    kernels = {
        "cfg2": rice + ": one launch per step",
        "cfg2s": ("airs::rice_kernel<DIFF,STREAM> (enc_rice.hip: 16 Ki-sample segments, no header): one launch "
                  "per step, one look-back chain of 4096 segments"),
        "cfg3": ("airs::rice_kernel<DIFF,AUTO> (enc_rice.hip: the per-frame Rice k chosen in-kernel from a "
                 "histogram of the samples in registers, the frame's segments meeting at a candidate barrier "
                 "instead of a look-back; then the Rice kernel's codeword pairs and arena): one launch per step"),
        "cfg4": rice + ": one launch per step",
        "cfg5": "airs::walk_ctx_kernel<4,DIFF,ZERO,Rice,MULTI,Rice,4> (enc_walk.hip): ONE launch per step, one "
                "1024-thread workgroup per stream walks its 16 acquisitions, the model in registers",
        "cfg5s8": "airs::walk_kernel<4,DIFF,ZERO,Rice,MULTI,Rice,%d> (enc_walk.hip, the segment walk): ONE launch "
                  "per step, a 320-thread workgroup per (stream, %d-sample segment) walks the 16 acquisitions, each "
                  "acquisition's look-back resolved one step later" %
                  (8, 2048),
        "cfg5fbs8": "airs::walk_kernel<4,DIFF,ZERO,Rice,MULTI,Rice,8> (the segment walk of cfg5s8) with the raw "
                    "frame size as capacity: ONE launch per step, then one read-back of the frame statuses and the "
                    "identifier patch (patch_ids_kernel); a context with a frame that does not fit would run again on "
                    "the device state machine (none in this data)",
        "cfg5fb": "airs::walk_ctx_kernel<4,DIFF,ZERO,Rice,MULTI,Rice,4> with the uncompressed fallback resolved on "
                  "the chip: ONE launch per step, then one read-back of the draw counts and the identifier patch "
                  "(patch_ids_kernel)",
    }
    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(wl)
            except Exception as e:  # report, never hide
                cpu = dict(error=repr(e))
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": wl["kind"],
            "data": (f"synthetic (counter-hash generator, SURVEY.md 8(d)), resident in HBM, rotated over {len(sets)} "
                     f"buffer sets ({sum(s.nbytes for s in sets) / 2**20:.0f} MiB > the 256 MiB Infinity Cache): "
                     f"cold reads"),
            "config": {
                "workload": wl["desc"],
                "name": wname,
                "frames_per_gpu": nf,
                "samples_per_frame": n,
                "sample_type": wl["kind"],
                "params": wl["params"],
                "auto_rice": bool(wl.get("auto_rice")),
                "parallelism": (f"{'streams' if wl['layout'] == 'streams' else 'frames'} sharded over {world} "
                                f"GPU(s) ({wl['layout']}), no data-path collective"),
                "compression_ratio": round(comp_bytes / (nf * 2 * n), 4),
            },
            "bitexact_vs_reference": bitexact,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernels[wname],
                "algorithmic_bytes_per_launch": alg_bytes,
                "algorithmic_bytes_note": "compulsory HBM reads of one step: 2 B/sample (u16), 4 B/sample "
                                          "(i16-in-i32), +2 B/sample model read per MODEL pass (SURVEY 8(d))",
                "avg_launch_ms_hip_events": round(kern_avg_ms, 5),
                "launch_us": launch_us,
                **({"frac_samples_only": round(in_bytes_rank / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "frac_samples_only_note": "the same launches against the sample bytes alone (4 B/sample): "
                                              "the model stays on the chip between acquisitions, so its 2 B/sample "
                                              "per MODEL pass are not re-read from HBM"}
                   if wl["params"].get("secondary_preprocessing") == MODEL else {}),
                "avg_launch_note": "HIP events around the K back-to-back steps on the engine stream, / K "
                                   "(all launches of a step)",
            },
            "cpu_baseline": cpu,
        }
        if warm:
            result["warm"] = warm
        if scaling_ref:
            if world > 1:
                scaling_ref["efficiency"] = round(value / (world * scaling_ref["value"]), 4)
                scaling_ref["efficiency_note"] = "value / (n_gpus x the one-GPU rate of the same per-GPU work)"
            result["scaling_reference"] = scaling_ref
        if gather:
            result["gather"] = gather
        print(json.dumps(result), flush=True)
    barrier()
    del sets
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
