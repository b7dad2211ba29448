#!/usr/bin/env python3
"""bench.py -- AIRSPACE encode throughput on MI355X.

One step = one cmp_gpu_compress() call over this rank's batch of frames whose
samples are already resident in HBM (BASELINE.json metric: encode GB/s on the
uncompressed input, 1 GB = 1e9 B, bit-exact vs the CPU reference).

  N = 1 (default)   configs[1]: 64 Mi u16 samples as 16 frames x 4 Mi
                    (the 24-bit header size field caps a frame at 8 388 607
                    samples), DIFF + GOLOMB_ZERO g = 32
  N > 1             configs[3] sharded round-robin: rank r encodes frames
                    f = r + N*j, j < 1024, of 64 Ki u16 samples (weak scaling:
                    128 MiB per GPU, so N = 8 is the 8192-frame config); the
                    compressed frames are then gathered to rank 0 over RCCL
                    (timed separately, not part of `value`)

Prints ONE JSON line on rank 0.  Diagnostics go to stderr.
"""
import argparse
import ctypes
import hashlib
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "airs-compression_amd")
METRIC = "encode GB/s (uncompressed in) on 16-bit frames; bit-exact vs CPU ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "airs_compression_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["airs_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


WORKLOADS = {
    "cfg2": dict(desc="configs[1]: 64 Mi u16 samples as 16 frames x 4 Mi, DIFF + GOLOMB_ZERO g=32",
                 n=4 << 20, frames=16, seed=0xA1A6, W=32, golden="cfg2_64Mi", layout="block"),
    "cfg4": dict(desc="configs[3]: frames of 64 Ki u16, round-robin over GPUs (1024 per GPU), "
                      "DIFF + GOLOMB_ZERO g=32",
                 n=64 << 10, frames=1024, seed=0xA1A8, W=32, golden="cfg4_8192", layout="roundrobin"),
}
PARAMS = dict(primary_preprocessing=1, primary_encoder_type=1, primary_encoder_param=32)


def measured_traffic(wname):
    """HBM bytes per launch of the encode kernel from the latest committed
    PMC passes (profiles/rNN_traffic_<workload>.json, written by
    scripts/traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE runs of this
    bench command), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_traffic_{wname}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        t = json.load(f)
    return t.get("traffic_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def frame_ids(wl, rank, world):
    if wl["layout"] == "roundrobin":
        return [rank + world * j for j in range(wl["frames"])]
    return [rank * wl["frames"] + j for j in range(wl["frames"])]


def cpu_baseline(wl, threads):
    """The reference's own CPU path (oracle/_ref/libref.so, compiled from the
    reference sources) timed on this host: OpenMP over frames, one context per
    thread.  Falls back to the clean-room port (oracle/liborc.so)."""
    api = sys.modules["airs_compression_amd"].cmpapi
    ref = os.path.join(ROOT, "oracle", "_ref", "libref.so")
    orc = os.path.join(ROOT, "oracle", "liborc.so")
    path, kind = (ref, "reference") if os.path.exists(ref) else (orc, "port")
    gen = ctypes.CDLL(orc, mode=ctypes.RTLD_LOCAL)
    gen.orc_synth_u16.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    n = wl["n"]
    nf = min(wl["frames"], 64)
    data = np.empty((nf, n), dtype=np.uint16)
    for j, f in enumerate(frame_ids(wl, 0, 1)[:nf]):
        gen.orc_synth_u16(wl["seed"], f, n, wl["W"], data[j].ctypes.data)
    drv = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    drv.drv_run.restype = ctypes.c_uint64
    lib = api.CmpLib(path)
    cap = lib.compress_bound(2 * n)
    cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
    stride = (cap + 7) // 8 * 8
    dst = api.aligned_empty(stride * nf)
    sizes = np.zeros(nf, dtype=np.uint32)
    prm = api.CmpParams(**PARAMS)

    def run(th):
        t0 = time.perf_counter()
        tot = drv.drv_run(ctypes.byref(prm), 0, ctypes.c_void_p(data.ctypes.data), ctypes.c_uint32(2 * n),
                          ctypes.c_uint64(2 * n), ctypes.c_uint32(nf), ctypes.c_uint32(1),
                          ctypes.c_void_p(dst.ctypes.data), ctypes.c_uint64(stride), ctypes.c_uint32(cap),
                          ctypes.c_void_p(sizes.ctypes.data), ctypes.c_int(th), ctypes.c_int(1))
        dt = time.perf_counter() - t0
        assert tot != 2**64 - 1
        return dt

    run(threads)  # warm-up
    times = sorted(run(threads) for _ in range(5))
    best = times[0]
    single = run(1) if nf <= 16 else None
    nbytes = nf * 2 * n
    out = dict(value=round(nbytes / best / 1e9, 4), unit="GB/s", cores=threads, kind=kind,
               sample=f"{nf} frames x {n} u16 samples ({nbytes / 2**20:.0f} MiB, the same synthetic frames "
                      f"and parameters), best of 5 after a warm-up, OpenMP over frames, one context per "
                      f"thread; host has {os.cpu_count()} logical CPUs",
               median_value=round(nbytes / times[2] / 1e9, 4))
    if single is not None:
        out["single_thread_value"] = round(nbytes / single / 1e9, 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
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

    wname = args.workload or ("cfg2" if world == 1 else "cfg4")
    wl = WORKLOADS[wname]
    n, nf = wl["n"], wl["frames"]
    fids = frame_ids(wl, rank, world)
    stride = 2 * n
    src = torch.empty(nf * stride, dtype=torch.uint8, device="cuda")
    if wl["layout"] == "block":
        assert eng.synthesize(src.data_ptr(), 2, wl["seed"], fids[0], n, nf, stride, wl["W"]) == 0
    else:
        for j, f in enumerate(fids):
            assert eng.synthesize(src.data_ptr() + j * stride, 2, wl["seed"], f, n, 1, stride, wl["W"]) == 0
    cap = lib.compress_bound(2 * n)
    cap = cap if not api.is_error(cap) else 3 * 2 * n + 64
    dstride = (cap + 7) // 8 * 8
    dst = torch.empty(nf * dstride, dtype=torch.uint8, device="cuda")
    sizes = torch.zeros(nf, dtype=torch.int32, device="cuda")
    ctxs = pkg.context_array(1)
    prm = api.CmpParams(**PARAMS)
    assert not api.is_error(lib.initialise(ctxs[0], prm))

    def step():
        r = eng.compress(ctxs, nf, "u16", src.data_ptr(), stride, stride, dst.data_ptr(), dstride, cap,
                         sizes.data_ptr())
        if r:
            raise RuntimeError("cmp_gpu_compress: " + api.error_name(r))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # one HIP event pair around the K launches (on the engine's stream): a
    # pair per launch would itself add ~8 us of stream time per step
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    kern_avg_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([wall], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())

    # ---- bit-exactness against the reference's golden digests -------------
    sz = sizes.cpu().numpy().astype(np.uint32)
    errs = [api.error_name(int(s)) for s in sz if api.is_error(int(s))]
    if errs:
        raise RuntimeError(f"frame errors: {errs[:4]}")
    host = dst.cpu().numpy()
    h = hashlib.sha256()
    for j in range(nf):
        b = bytearray(host[j * dstride:j * dstride + int(sz[j])])
        b[8:14] = b"\0" * 6
        h.update(b)
    digest = h.hexdigest()
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        gold = json.load(f)["configs"][wl["golden"]]
    key = f"shard_digests_n{world}" if wl["layout"] == "roundrobin" else None
    if key and key in gold:
        want = gold[key][rank]
    elif wl["layout"] == "block" and rank == 0:
        want = gold["digest"]
    else:
        want = None
    bitexact = (digest == want) if want else None
    comp_bytes = int(sz.astype(np.uint64).sum())

    # ---- gather of compressed frames to rank 0 over RCCL (not in `value`) --
    gather = None
    if world > 1 and not args.no_gather:
        layout = "roundrobin" if wl["layout"] == "roundrobin" else "block"
        gather, g = pkg.shard.gather_frames_timed(dist, dst, dstride, sizes, nf, rank, world, layout=layout,
                                                  patch_base=0)
        if g is not None:
            host_all = g.data.cpu().numpy()
            offs, lens = g.offsets.numpy(), g.sizes.numpy()
            hg = hashlib.sha256()
            for f in range(g.num_frames):
                b = bytearray(host_all[offs[f]:offs[f] + lens[f]])
                ok_id = int.from_bytes(b[8:14], "big") == 1 + f
                b[8:14] = b"\0" * 6
                hg.update(b)
                if not ok_id:
                    gather["identifier_patch_ok"] = False
            gather.setdefault("identifier_patch_ok", True)
            gwant = gold.get(f"gather_digest_n{world}") if wl["layout"] == "roundrobin" else None
            gather["bitexact_vs_reference"] = (hg.hexdigest() == gwant) if gwant else None
            del g, host_all

    in_bytes_rank = nf * 2 * n
    total_in = in_bytes_rank * world
    value = total_in * args.steps / wall_max / 1e9
    ms_step = wall_max / args.steps * 1e3
    traffic, traffic_src = measured_traffic(wname)
    achieved = in_bytes_rank / (kern_avg_ms * 1e-3) / 1e9
    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                cpu = cpu_baseline(wl, threads=min(16, os.cpu_count() or 1))
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
            "dtype": "u16",
            "data": "synthetic (counter-hash generator, SURVEY.md 8(d)), resident in HBM",
            "config": {
                "workload": wl["desc"],
                "frames_per_gpu": nf,
                "samples_per_frame": n,
                "preprocessing": "DIFF", "encoder": "GOLOMB_ZERO", "golomb_g": 32,
                "parallelism": f"frames sharded over {world} GPU(s), no data-path collective",
                "compression_ratio": round(comp_bytes / in_bytes_rank, 4),
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
                "kernel": "airs::encode_kernel<2,1,1,true> (u16, DIFF, GOLOMB_ZERO, Rice)",
                "algorithmic_bytes_per_launch": in_bytes_rank,
                "avg_launch_ms_hip_events": round(kern_avg_ms, 5),
                "avg_launch_note": "HIP events around the K back-to-back launches on the engine stream, / K",
            },
            "cpu_baseline": cpu,
        }
        if gather:
            result["gather"] = gather
        print(json.dumps(result), flush=True)
    barrier()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
