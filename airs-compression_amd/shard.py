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
  2. every rank compacts its frames into one contiguous buffer (frame j of the
     rank at the exclusive prefix sum of the sizes);
  3. the root posts one receive per peer and every peer one send (RCCL has no
     gatherv; point-to-point maps onto the direct xGMI link between the pair);
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
    """Global frame numbers owned by `rank`."""
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


def compact(dst: torch.Tensor, dst_stride: int, sizes: torch.Tensor, num_frames: int) -> torch.Tensor:
    """Concatenate frames j < num_frames (frame j at dst[j*dst_stride:] with
    sizes[j] bytes) into one contiguous uint8 tensor on dst's device."""
    if num_frames == 0:
        return dst.new_empty(0)
    d2 = dst[:num_frames * dst_stride].view(num_frames, dst_stride)
    lens = sizes[:num_frames].to(torch.int64)
    keep = torch.arange(dst_stride, device=dst.device)[None, :] < lens[:, None]
    return d2[keep]


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

    def patch_identifiers(self, base: int) -> None:
        """Write identifier base + 1 + f (48-bit big-endian, header bytes
        8..13) into every frame."""
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
                  group=None) -> GatheredFrames | None:
    """Gather every rank's compressed frames on `root` (steps 1-4 above).
    Returns the GatheredFrames on the root, None elsewhere.  All ranks must
    hold the same num_frames."""
    local_sizes = sizes[:num_frames].to(torch.int32).contiguous()
    all_sizes = [torch.empty_like(local_sizes) for _ in range(world)]
    dist.all_gather(all_sizes, local_sizes, group=group)
    table = torch.stack(all_sizes).cpu().to(torch.int64)  # [world, F]
    _check_sizes(table.reshape(-1))

    buf = compact(dst, dst_stride, local_sizes, num_frames)
    totals = table.sum(dim=1).tolist()
    if rank != root:
        if totals[rank]:
            dist.send(buf, dst=root, group=group)
        return None

    parts = []
    reqs = []
    for r in range(world):
        if r == root:
            parts.append(buf)
            continue
        t = torch.empty(int(totals[r]), dtype=torch.uint8, device=dst.device)
        if totals[r]:
            reqs.append(dist.irecv(t, src=r, group=group))
        parts.append(t)
    for q in reqs:
        q.wait()
    data = torch.cat(parts) if world > 1 else buf

    base = torch.tensor([0] + totals[:-1], dtype=torch.int64).cumsum(0)   # rank offsets in data
    within = torch.cumsum(table, dim=1) - table                            # frame offsets in rank buf
    off_rank = base[:, None] + within                                      # [world, F]
    nf_total = world * num_frames
    fid = torch.stack([global_frame_ids(num_frames, r, world, layout) for r in range(world)])
    offsets = torch.empty(nf_total, dtype=torch.int64)
    fsizes = torch.empty(nf_total, dtype=torch.int64)
    offsets[fid.reshape(-1)] = off_rank.reshape(-1)
    fsizes[fid.reshape(-1)] = table.reshape(-1)
    return GatheredFrames(data=data, offsets=offsets, sizes=fsizes)


def gather_frames_timed(dist, dst, dst_stride, sizes, num_frames, rank, world, root: int = 0,
                        layout: str = "roundrobin", patch_base: int | None = 0):
    """gather_frames between two barriers, timed on the host clock (device
    work synchronised).  Returns (stats dict, GatheredFrames or None)."""
    cuda = dst.is_cuda

    def sync():
        if cuda:
            torch.cuda.synchronize()

    sync()
    dist.barrier()
    t0 = time.perf_counter()
    g = gather_frames(dist, dst, dst_stride, sizes, num_frames, rank, world, root=root, layout=layout)
    if g is not None and patch_base is not None:
        g.patch_identifiers(patch_base)
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
                     note="all_gather(sizes) + compaction + point-to-point sends to the root + "
                          "identifier patch; peak = one direct xGMI link per peer")
    return stats, g


def compact_bytes_of(g: GatheredFrames, rank: int, world: int, num_frames: int, layout: str) -> int:
    """Bytes of `rank`'s own frames inside a GatheredFrames."""
    fid = global_frame_ids(num_frames, rank, world, layout)
    return int(g.sizes[fid].sum())
