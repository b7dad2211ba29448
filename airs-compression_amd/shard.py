"""Frame and stream sharding over the GPUs of a node and the gather of the
compressed frames to one rank.

The units of the encode path are independent: a frame (lib/compress/cmp.c:396-407
compresses one frame per call) or, when frames carry state from one to the
next (a MODEL secondary pass reads the model the previous frame left,
cmp.c:250-254, 304-311), a stream: one context's frames in acquisition order.
So the data path needs no collective: rank r encodes its own units with
cmp_gpu_compress and the node only exchanges the finished bitstreams.

Layouts (global frame g, rank r of N, F frames per rank):
  "roundrobin"  frame g on rank g mod N (local frame j = g // N)
  "block"       frames r*F .. r*F + F-1 on rank r
  "streams"     streams of `fpc` frames, stream s on rank s mod N: local frame
                i*fpc + a is global frame s*fpc + a with s = r + N*i (BASELINE
                config 5: each model stays on one GPU)

Gather protocol (one process per GPU, torch.distributed; backend "nccl" is
RCCL over xGMI on the MI355X node, "gloo" on CPU for the tests):

  1. all_gather of one int64 per frame: the compressed size (or error value)
     and, in bits 32-39, the number of timestamp-callback draws the frame made
     (cmp_gpu_batch.draws: 0, 1 per reset, 2 or 3 for a fallback);
  2. every rank packs its frames back to back (8-byte aligned offsets, the
     exclusive prefix sum of the rounded sizes: cmp_gpu_pack_frames on the
     GPU, reading only the compressed bytes);
  3. the root posts one receive per peer straight into its slice of the
     node buffer and every peer one send, as one batch_isend_irecv group
     (RCCL has no gatherv; grouped point-to-point maps onto the direct xGMI
     link between each pair);
  4. the root builds the frame table in global frame order and, on request,
     rewrites the 48-bit header identifiers (bytes 8..13,
     lib/common/header.c:60-62) to those ONE process would have drawn for the
     node's frames in global order with the default counter: frame g gets
     base + (inclusive scan of the draws in global order)[g].  For the frame
     layouts that is one context compressing every frame in order (exact
     when no frame depends on the frame before it: no secondary passes; the
     uncompressed fallback is fine); for "streams" it is one batch over all
     the streams' contexts in stream order.  Frames before the first draw of
     their stream keep the identifier they carry.

Works on CUDA (HIP) and CPU tensors alike; nothing here touches the oracle.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

XGMI_LINK_GBS = 153.0  # per direct link, MI355X_MICROARCH.md
LAYOUTS = ("roundrobin", "block", "streams")


def rank_frames(num_frames: int, rank: int, world: int, layout: str = "roundrobin", fpc: int = 1) -> list[int]:
    """Global frame numbers owned by `rank`, in local order.  "block" and
    "streams" give every rank the same count: frames (streams) beyond the last
    whole round belong to no rank (callers size num_frames to a multiple)."""
    if layout == "roundrobin":
        return list(range(rank, num_frames, world))
    if layout == "streams":
        nstreams = num_frames // fpc
        return [s * fpc + a for s in range(rank, nstreams - nstreams % world, world) for a in range(fpc)]
    per = num_frames // world
    return list(range(rank * per, (rank + 1) * per))


def global_frame_ids(frames_per_rank: int, rank: int, world: int, layout: str, fpc: int = 1) -> torch.Tensor:
    j = torch.arange(frames_per_rank, dtype=torch.int64)
    if layout == "roundrobin":
        return rank + world * j
    if layout == "streams":
        return (rank + world * (j // fpc)) * fpc + j % fpc
    return rank * frames_per_rank + j


def _check_sizes(sizes: torch.Tensor) -> None:
    # cmp error values are (uint32)-code, code < 128 (lib/common/cmp_errors.h):
    # as int32 they are the range [-127, -1]
    flat = sizes.reshape(-1)
    bad = torch.nonzero(flat < 0)
    if bad.numel():
        idx = int(bad[0, 0])
        raise RuntimeError(f"frame slot {idx} carries error value {int(flat[idx]) & 0xFFFFFFFF:#x}, not a size")


def packed_offsets(sizes: torch.Tensor) -> torch.Tensor:
    """Offsets of frames packed back to back at 8-byte aligned offsets
    (int64, one more than frames: the last is the total).  Error values take
    no bytes.  The same rule as cmp_gpu_pack_frames (include/cmp_gpu.h)."""
    s = sizes.to(torch.int64).reshape(-1)
    lens = torch.where(s < 0, torch.zeros_like(s), (s + 7) // 8 * 8)
    out = torch.zeros(s.numel() + 1, dtype=torch.int64, device=s.device)
    out[1:] = torch.cumsum(lens, 0)
    return out


def _check_engine_stream(engine) -> None:
    """The packing runs on the engine's stream, while its inputs, output and
    temporaries are ordered on torch's current stream: they must be the same
    stream."""
    cur = torch.cuda.current_stream().cuda_stream
    eng = engine.stream or 0
    if eng != cur:
        raise RuntimeError(f"engine stream {eng:#x} is not torch's current stream {cur:#x}; create the engine "
                           f"with torch.cuda.current_stream().cuda_stream")


def pack(dst: torch.Tensor, dst_stride: int, sizes: torch.Tensor, num_frames: int, out: torch.Tensor,
         engine=None, frame_capacity: int | None = None, total: int | None = None) -> int:
    """Pack frames j < num_frames (frame j at dst[j*dst_stride:], sizes[j]
    bytes) into `out` at packed_offsets(sizes).  On the GPU this is one
    cmp_gpu_pack_frames call on the engine's stream (a scan and a copy kernel
    that read only the compressed bytes; the engine must run on torch's
    current stream); on the CPU one slice copy per frame.  `total` (the packed
    size, when the caller knows it) spares a read-back of the sizes.  Returns
    the bytes read from dst (= the packed size)."""
    if num_frames == 0:
        return 0
    if engine is not None and dst.is_cuda:
        _check_engine_stream(engine)
        if total is None:
            total = int(packed_offsets(sizes[:num_frames])[-1])
        assert out.numel() >= total and out.dtype == torch.uint8
        sz = sizes[:num_frames].to(torch.int32).contiguous()
        d_offs = torch.empty(num_frames + 1, dtype=torch.int64, device=dst.device)
        cap = frame_capacity if frame_capacity is not None else dst_stride
        r = engine.pack_frames(dst.data_ptr(), dst_stride, cap, sz.data_ptr(), num_frames, out.data_ptr(),
                               d_offs.data_ptr())
        if r:
            raise RuntimeError(f"cmp_gpu_pack_frames failed: {r:#x}")
        # sz and d_offs were allocated on the current stream, which is the
        # engine's: their memory is only reused by work queued after the pack
        return total
    o = packed_offsets(sizes[:num_frames].cpu()).tolist()
    assert out.numel() >= o[-1] and out.dtype == torch.uint8
    for j in range(num_frames):
        n8 = o[j + 1] - o[j]
        if n8:
            out[o[j]:o[j] + n8].copy_(dst[j * dst_stride:j * dst_stride + n8])
    return o[-1]


def check_patchable(params, draws, layout: str = "roundrobin") -> None:
    """Raise ValueError unless the identifier patch of step 4 is exact.

    Without per-frame draw counts every frame is taken to make one draw (a
    primary pass that cannot fall back), which `params` must guarantee.  With
    draw counts the fallback is fine (its extra draws are counted), but for
    the frame layouts a frame must still not depend on the frame before it:
    a secondary pass on one rank followed the previous frame of THAT rank's
    context, not the previous global frame, so its identifier (and its bytes)
    are not what one context over all frames would give.  So for
    "roundrobin" and "block" secondary passes are refused, by the parameters
    and by any frame that made no draw (a secondary pass draws nothing,
    cmp.c:228-248).  "streams" keep every stream on one rank, so draws are
    exact there."""
    if draws is None:
        if params is None or getattr(params, "secondary_iterations", 0) or \
                getattr(params, "uncompressed_fallback_enabled", 0):
            raise ValueError("identifier patching without per-frame draw counts needs secondary_iterations == 0 "
                             "and the fallback disabled: pass the draws cmp_gpu_compress reports "
                             "(cmp_gpu_batch.draws)")
        return
    if layout == "streams":
        return
    if params is not None and getattr(params, "secondary_iterations", 0):
        raise ValueError(f"identifier patching of the {layout!r} layout needs secondary_iterations == 0 (a "
                         f"secondary pass depends on its rank's previous frame); use the 'streams' layout")
    d = torch.as_tensor(draws)
    if d.numel() and bool((d.reshape(-1) == 0).any()):
        raise ValueError(f"identifier patching of the {layout!r} layout: a frame made no identifier draw (a "
                         f"secondary pass, which depends on its rank's previous frame); use the 'streams' layout")


def check_patchable_all(dist, params, draws, layout: str, device, group=None) -> None:
    """check_patchable on every rank, decided together: each rank
    checks its own draws and parameters, and one all_reduce(MAX) of the
    refusal flag makes every rank raise if any rank refuses, so no rank is
    left waiting in a barrier or the gather while a peer has raised."""
    err = None
    try:
        check_patchable(params, draws, layout)
    except ValueError as e:
        err = e
    flag = torch.tensor([1 if err is not None else 0], dtype=torch.int32, device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    if int(flag.item()):
        raise err if err is not None else ValueError(
            f"identifier patching of the {layout!r} layout refused on another rank (its draw counts show a "
            f"secondary pass, or its parameters do); use the 'streams' layout")


def assign_identifiers(draws: torch.Tensor, base: int, layout: str, fpc: int = 1) -> tuple[torch.Tensor, torch.Tensor]:
    """Identifiers of frames in global order from their draw counts (int64,
    global order): (ids, keep) with ids[g] = base + inclusive scan of the
    draws, and keep[g] True where the frame made no draw yet in its context
    (it carries the identifier it has; for the frame layouts the context is
    the whole sequence, for "streams" the stream).  The reference's process-
    global counter: lib/compress/cmp.c:27-50, 438-449."""
    d = draws.to(torch.int64).reshape(-1)
    ids = (base + torch.cumsum(d, 0)) & ((1 << 48) - 1)
    unit = fpc if layout == "streams" else d.numel()
    per = torch.cumsum(d.reshape(-1, unit), 1).reshape(-1)
    return ids, per == 0


@dataclass
class GatheredFrames:
    """Compressed frames of the whole node on the root, in global frame order.

    `data` holds the peers' compacted buffers back to back (rank order);
    frame f occupies data[offsets[f] : offsets[f] + sizes[f]].  `draws` (if
    the ranks passed them) is each frame's identifier-draw count."""
    data: torch.Tensor
    offsets: torch.Tensor  # int64 [num_frames], in f order (on data's device)
    sizes: torch.Tensor    # int64 [num_frames], in f order (host)
    draws: torch.Tensor | None = None  # int64 [num_frames], in f order (host)
    layout: str = "roundrobin"
    fpc: int = 1

    @property
    def num_frames(self) -> int:
        return int(self.sizes.numel())

    def frame(self, f: int) -> torch.Tensor:
        o = int(self.offsets[f])
        return self.data[o:o + int(self.sizes[f])]

    def ordered(self) -> torch.Tensor:
        """One contiguous stream of all frames in f order (a copy)."""
        if self.num_frames == 0:
            return self.data[:0]
        return torch.cat([self.frame(f) for f in range(self.num_frames)])

    def patch_identifiers(self, base: int, params=None) -> None:
        """Rewrite header bytes 8..13 of every frame that is not an error
        with the identifier one process would have drawn (module docstring,
        step 4), on the data's device.  Without gathered draw counts every
        frame counts one draw, which `params` must guarantee
        (check_patchable)."""
        check_patchable(params, self.draws, self.layout)
        if self.num_frames == 0:
            return
        dev = self.data.device
        draws = self.draws if self.draws is not None else torch.ones(self.num_frames, dtype=torch.int64)
        ids, keep = assign_identifiers(draws, base, self.layout, self.fpc)
        write = (~keep) & (self.sizes >= 14)
        ids = ids[write].to(dev)
        offs = self.offsets.to(dev)[write.to(dev)]
        sh = 8 * (5 - torch.arange(6, dtype=torch.int64, device=dev))
        val = ((ids[:, None] >> sh[None, :]) & 0xFF).to(torch.uint8)
        pos = offs[:, None] + 8 + torch.arange(6, dtype=torch.int64, device=dev)[None, :]
        self.data[pos.reshape(-1)] = val.reshape(-1)


def gather_frames(dist, dst: torch.Tensor, dst_stride: int, sizes: torch.Tensor, num_frames: int,
                  rank: int, world: int, root: int = 0, layout: str = "roundrobin",
                  group=None, engine=None, frame_capacity: int | None = None,
                  stats: dict | None = None, draws=None, fpc: int = 1) -> GatheredFrames | None:
    """Gather every rank's compressed frames on `root` (steps 1-4 above).
    Returns the GatheredFrames on the root, None elsewhere.  All ranks must
    hold the same num_frames (a multiple of fpc for "streams").  `engine` (a
    GpuEngine on torch's current stream) packs on the device; without it
    (CPU tensors, gloo) the packing is one slice copy per frame.  `draws`:
    this rank's per-frame identifier draws (cmp_gpu_batch.draws), optional.

    The size table is the one host read-back (the receives are sized from
    it); offsets, identifiers and the header patch stay on the data's device.
    The root's buffer holds every rank's packed frames back to back; each peer
    is received straight into its slice (no concatenation), and the
    transfers are posted as one batch (batch_isend_irecv: grouped
    point-to-point, one direct xGMI link per peer under RCCL)."""
    assert layout in LAYOUTS
    if layout == "streams":
        assert fpc >= 1 and num_frames % fpc == 0
    local = sizes[:num_frames].to(torch.int64) & 0xFFFFFFFF
    if draws is not None:
        d = torch.as_tensor(draws[:num_frames], dtype=torch.int64).to(local.device)
        local = local | (d << 32)
    local = local.contiguous()
    gathered = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(gathered, local, group=group)
    table64 = torch.stack(gathered).cpu()  # [world, F]: the one host read-back
    table = (table64 & 0xFFFFFFFF).to(torch.int32).to(torch.int64)  # sign-extended error values
    _check_sizes(table.reshape(-1))
    poffs = [packed_offsets(table[r]) for r in range(world)]
    totals = [int(p[-1]) for p in poffs]
    base = [0]
    for t in totals[:-1]:
        base.append(base[-1] + t)

    if rank != root:
        buf = torch.empty(totals[rank], dtype=torch.uint8, device=dst.device)
        nread = pack(dst, dst_stride, sizes, num_frames, buf, engine, frame_capacity, total=totals[rank])
        if stats is not None:
            stats["pack_bytes_read"] = nread
        if totals[rank]:
            for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, buf, root, group=group)]):
                q.wait()
        return None

    data = torch.empty(sum(totals), dtype=torch.uint8, device=dst.device)
    ops = [dist.P2POp(dist.irecv, data[base[r]:base[r] + totals[r]], r, group=group)
           for r in range(world) if r != root and totals[r]]
    reqs = dist.batch_isend_irecv(ops) if ops else []
    nread = pack(dst, dst_stride, sizes, num_frames, data[base[root]:base[root] + totals[root]], engine,
                 frame_capacity, total=totals[root])
    if stats is not None:
        stats["pack_bytes_read"] = nread
    for q in reqs:
        q.wait()

    off_rank = torch.stack([torch.tensor(base[r], dtype=torch.int64) + poffs[r][:-1] for r in range(world)])
    nf_total = world * num_frames
    fid = torch.stack([global_frame_ids(num_frames, r, world, layout, fpc) for r in range(world)]).reshape(-1)
    offsets = torch.empty(nf_total, dtype=torch.int64)
    fsizes = torch.empty(nf_total, dtype=torch.int64)
    offsets[fid] = off_rank.reshape(-1)
    fsizes[fid] = table.reshape(-1)
    fdraws = None
    if draws is not None:
        fdraws = torch.empty(nf_total, dtype=torch.int64)
        fdraws[fid] = (table64 >> 32).reshape(-1)
    return GatheredFrames(data=data, offsets=offsets.to(data.device), sizes=fsizes, draws=fdraws, layout=layout,
                          fpc=fpc)


def gather_frames_timed(dist, dst, dst_stride, sizes, num_frames, rank, world, root: int = 0,
                        layout: str = "roundrobin", patch_base: int | None = None, params=None, engine=None,
                        frame_capacity: int | None = None, draws=None, fpc: int = 1):
    """gather_frames (and, with patch_base, the identifier patch) between two
    barriers, timed on the host clock (device work synchronised).  Returns
    (stats dict, GatheredFrames or None)."""
    cuda = dst.is_cuda
    if patch_base is not None:
        # on every rank, before any other communication, decided together
        check_patchable_all(dist, params, draws, layout, dst.device)

    def sync():
        if cuda:
            torch.cuda.synchronize()

    sync()
    dist.barrier()
    t0 = time.perf_counter()
    pstats = {}
    g = gather_frames(dist, dst, dst_stride, sizes, num_frames, rank, world, root=root, layout=layout,
                      engine=engine, frame_capacity=frame_capacity, stats=pstats, draws=draws, fpc=fpc)
    if g is not None and patch_base is not None:
        g.patch_identifiers(patch_base, params)
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dst.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    stats = None
    if g is not None:
        ingress = int(g.data.numel()) - int(compact_bytes_of(g, root, world, num_frames, layout, fpc))
        peak = XGMI_LINK_GBS * max(world - 1, 1)
        stats = dict(gather_ms=round(dt * 1e3, 4), frames=g.num_frames, bytes_total=int(g.data.numel()),
                     root_ingress_bytes=ingress, ingress_GBs=round(ingress / dt / 1e9, 2) if dt > 0 else None,
                     xgmi_peak_GBs=peak, frac_of_xgmi=round(ingress / dt / 1e9 / peak, 4) if dt > 0 else None,
                     root_pack_bytes_read=pstats.get("pack_bytes_read"), layout=layout,
                     packing="cmp_gpu_pack_frames (device)" if engine is not None and dst.is_cuda else
                             "slice copies (host)",
                     identifiers=("patched from the gathered draw counts" if draws is not None else
                                  "patched, one draw per frame") if patch_base is not None else "as encoded",
                     note="all_gather(sizes | draws) + packing (8-byte aligned frames, compressed bytes only) + "
                          "batched point-to-point receives into the root buffer + identifier patch; peak = "
                          "one direct xGMI link per peer")
    return stats, g


def compact_bytes_of(g: GatheredFrames, rank: int, world: int, num_frames: int, layout: str, fpc: int = 1) -> int:
    """Packed bytes of `rank`'s own frames inside a GatheredFrames."""
    fid = global_frame_ids(num_frames, rank, world, layout, fpc)
    return int(packed_offsets(g.sizes[fid])[-1])
