"""Frame sharding over the GPUs of a node and the gather of the compressed
frames to one rank.

Frames are independent units of the encode path (lib/compress/cmp.c:396-407
compresses one frame per call, the only cross-frame state being the context's
sequence counter and model), so the data path needs no collective: rank r
encodes its own frames with cmp_gpu_compress and the node only exchanges the
finished bitstreams afterwards.

Gather protocol (one process per GPU, torch.distributed; backend "nccl" is
RCCL over xGMI on the MI355X node, "gloo" on CPU for the tests):

  1. all_gather of the per-frame compressed sizes (int32, error values
     included; 4 B per frame per rank);
  2. every rank packs its frames back to back (8-byte aligned offsets, the
     exclusive prefix sum of the rounded sizes: cmp_gpu_pack_frames on the
     GPU, reading only the compressed bytes);
  3. the root posts one receive per peer straight into its slice of the
     node buffer and every peer one send, as one batch_isend_irecv group
     (RCCL has no gatherv; grouped point-to-point maps onto the direct xGMI
     link between each pair);
  4. the root builds the frame table in global frame order f (round robin:
     f = r + N*j; block: f = r*F + j) and, on request, patches the 48-bit
     header identifiers (bytes 8..13, lib/common/header.c:60-62) to
     base + 1 + f, the sequence a single cmp_context would have produced with
     the default timestamp callback and fallback disabled.

Works on CUDA (HIP) and CPU tensors alike; nothing here touches the oracle.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

XGMI_LINK_GBS = 153.0  # per direct link, MI355X_MICROARCH.md


def rank_frames(num_frames: int, rank: int, world: int, layout: str = "roundrobin") -> list[int]:
    """Global frame numbers owned by `rank`.  "block" gives every rank
    num_frames // world consecutive frames: the last num_frames % world
    frames belong to no rank (callers size num_frames to a multiple)."""
    if layout == "roundrobin":
        return list(range(rank, num_frames, world))
    per = num_frames // world
    return list(range(rank * per, (rank + 1) * per))


def global_frame_ids(frames_per_rank: int, rank: int, world: int, layout: str) -> torch.Tensor:
    j = torch.arange(frames_per_rank, dtype=torch.int64)
    return rank + world * j if layout == "roundrobin" else rank * frames_per_rank + j


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


def pack(dst: torch.Tensor, dst_stride: int, sizes: torch.Tensor, num_frames: int, out: torch.Tensor,
         engine=None, frame_capacity: int | None = None) -> int:
    """Pack frames j < num_frames (frame j at dst[j*dst_stride:], sizes[j]
    bytes) into `out` at packed_offsets(sizes).  On the GPU this is one
    cmp_gpu_pack_frames call (a scan and a copy kernel that read only the
    compressed bytes); on the CPU one slice copy per frame.  Returns the
    bytes read from dst (= the packed size)."""
    if num_frames == 0:
        return 0
    offs = packed_offsets(sizes[:num_frames].cpu())
    total = int(offs[-1])
    assert out.numel() >= total and out.dtype == torch.uint8
    if engine is not None and dst.is_cuda:
        sz = sizes[:num_frames].to(torch.int32).contiguous()
        d_offs = torch.empty(num_frames + 1, dtype=torch.int64, device=dst.device)
        cap = frame_capacity if frame_capacity is not None else dst_stride
        r = engine.pack_frames(dst.data_ptr(), dst_stride, cap, sz.data_ptr(), num_frames, out.data_ptr(),
                               d_offs.data_ptr())
        if r:
            raise RuntimeError(f"cmp_gpu_pack_frames failed: {r:#x}")
        return total
    o = offs.tolist()
    for j in range(num_frames):
        n8 = o[j + 1] - o[j]
        if n8:
            out[o[j]:o[j] + n8].copy_(dst[j * dst_stride:j * dst_stride + n8])
    return total


def check_patchable(params) -> None:
    """Raise ValueError unless base + 1 + f are the identifiers of the frames
    (GatheredFrames.patch_identifiers)."""
    if params is None or getattr(params, "secondary_iterations", 0) or \
            getattr(params, "uncompressed_fallback_enabled", 0):
        raise ValueError("identifier patching needs secondary_iterations == 0 and the fallback disabled")


@dataclass
class GatheredFrames:
    """Compressed frames of the whole node on the root, in global frame order.

    `data` holds the peers' compacted buffers back to back (rank order);
    frame f occupies data[offsets[f] : offsets[f] + sizes[f]]."""
    data: torch.Tensor
    offsets: torch.Tensor  # int64 [num_frames], in f order
    sizes: torch.Tensor    # int64 [num_frames], in f order

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

    def patch_identifiers(self, base: int, params) -> None:
        """Write identifier base + 1 + f (48-bit big-endian, header bytes
        8..13) into every frame: the identifiers one context drawing with the
        default timestamp callback gives a frame sequence when every frame is
        a primary pass that cannot fall back (cmp.c:228-237: one reset, one
        draw per frame).  With secondary passes (frames of one reset cycle
        share an identifier) or the uncompressed fallback (three draws per
        fallback) that sequence depends on the outcomes, so those parameter
        sets are refused: params is the cmp_params the frames were made with."""
        check_patchable(params)
        if self.num_frames == 0:
            return
        dev = self.data.device
        ids = (base + 1 + torch.arange(self.num_frames, dtype=torch.int64)) & ((1 << 48) - 1)
        sh = 8 * (5 - torch.arange(6, dtype=torch.int64))
        val = ((ids[:, None] >> sh[None, :]) & 0xFF).to(torch.uint8)
        pos = self.offsets.cpu()[:, None] + 8 + torch.arange(6, dtype=torch.int64)[None, :]
        self.data[pos.reshape(-1).to(dev)] = val.reshape(-1).to(dev)


def gather_frames(dist, dst: torch.Tensor, dst_stride: int, sizes: torch.Tensor, num_frames: int,
                  rank: int, world: int, root: int = 0, layout: str = "roundrobin",
                  group=None, engine=None, frame_capacity: int | None = None,
                  stats: dict | None = None) -> GatheredFrames | None:
    """Gather every rank's compressed frames on `root` (steps 1-4 above).
    Returns the GatheredFrames on the root, None elsewhere.  All ranks must
    hold the same num_frames.  `engine` (a GpuEngine) packs on the device;
    without it (CPU tensors, gloo) the packing is one slice copy per frame.

    The root's buffer holds every rank's packed frames back to back; each peer
    is received straight into its slice (no concatenation), and the
    transfers are posted as one batch (batch_isend_irecv: grouped
    point-to-point, one direct xGMI link per peer under RCCL)."""
    local_sizes = sizes[:num_frames].to(torch.int32).contiguous()
    all_sizes = [torch.empty_like(local_sizes) for _ in range(world)]
    dist.all_gather(all_sizes, local_sizes, group=group)
    table = torch.stack(all_sizes).cpu().to(torch.int64)  # [world, F]
    _check_sizes(table.reshape(-1))
    poffs = [packed_offsets(table[r]) for r in range(world)]
    totals = [int(p[-1]) for p in poffs]
    base = [0]
    for t in totals[:-1]:
        base.append(base[-1] + t)

    if rank != root:
        buf = torch.empty(totals[rank], dtype=torch.uint8, device=dst.device)
        nread = pack(dst, dst_stride, local_sizes, num_frames, buf, engine, frame_capacity)
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
    nread = pack(dst, dst_stride, local_sizes, num_frames, data[base[root]:base[root] + totals[root]], engine,
                 frame_capacity)
    if stats is not None:
        stats["pack_bytes_read"] = nread
    for q in reqs:
        q.wait()

    off_rank = torch.stack([torch.tensor(base[r], dtype=torch.int64) + poffs[r][:-1] for r in range(world)])
    nf_total = world * num_frames
    fid = torch.stack([global_frame_ids(num_frames, r, world, layout) for r in range(world)])
    offsets = torch.empty(nf_total, dtype=torch.int64)
    fsizes = torch.empty(nf_total, dtype=torch.int64)
    offsets[fid.reshape(-1)] = off_rank.reshape(-1)
    fsizes[fid.reshape(-1)] = table.reshape(-1)
    return GatheredFrames(data=data, offsets=offsets, sizes=fsizes)


def gather_frames_timed(dist, dst, dst_stride, sizes, num_frames, rank, world, root: int = 0,
                        layout: str = "roundrobin", patch_base: int | None = 0, params=None, engine=None,
                        frame_capacity: int | None = None):
    """gather_frames between two barriers, timed on the host clock (device
    work synchronised).  Returns (stats dict, GatheredFrames or None)."""
    cuda = dst.is_cuda
    if patch_base is not None:
        check_patchable(params)  # on every rank, before any communication

    def sync():
        if cuda:
            torch.cuda.synchronize()

    sync()
    dist.barrier()
    t0 = time.perf_counter()
    pstats = {}
    g = gather_frames(dist, dst, dst_stride, sizes, num_frames, rank, world, root=root, layout=layout,
                      engine=engine, frame_capacity=frame_capacity, stats=pstats)
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
        ingress = int(g.data.numel()) - int(compact_bytes_of(g, root, world, num_frames, layout))
        peak = XGMI_LINK_GBS * max(world - 1, 1)
        stats = dict(gather_ms=round(dt * 1e3, 4), frames=g.num_frames, bytes_total=int(g.data.numel()),
                     root_ingress_bytes=ingress, ingress_GBs=round(ingress / dt / 1e9, 2) if dt > 0 else None,
                     xgmi_peak_GBs=peak, frac_of_xgmi=round(ingress / dt / 1e9 / peak, 4) if dt > 0 else None,
                     root_pack_bytes_read=pstats.get("pack_bytes_read"),
                     packing="cmp_gpu_pack_frames (device)" if engine is not None and dst.is_cuda else
                             "slice copies (host)",
                     note="all_gather(sizes) + packing (8-byte aligned frames, compressed bytes only) + "
                          "batched point-to-point receives into the root buffer + identifier patch; peak = "
                          "one direct xGMI link per peer")
    return stats, g


def compact_bytes_of(g: GatheredFrames, rank: int, world: int, num_frames: int, layout: str) -> int:
    """Packed bytes of `rank`'s own frames inside a GatheredFrames."""
    fid = global_frame_ids(num_frames, rank, world, layout)
    return int(packed_offsets(g.sizes[fid])[-1])
