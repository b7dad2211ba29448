"""cmp_gpu_gather_plan (the C multi-GPU gather's host plan, csrc/cmp_gather.c)
against shard.py's restatement of the same protocol: for
random all-gathered tables (sizes and identifier draws), every layout, 1 to 8
ranks: each rank's packed bytes, each global frame's offset in the root's
buffer and size, and the identifiers one process would have drawn
(assign_identifiers), plus the refusals (an error value; a frame layout with
a frame that made no draw).  Host only: no device, no RCCL."""
import numpy as np
import pytest
import torch

from conftest import load_pkg

pkg = load_pkg()
shard = pkg.shard
api = pkg.cmpapi
LAYOUTS = {"roundrobin": pkg.LAYOUT_ROUNDROBIN, "block": pkg.LAYOUT_BLOCK, "streams": pkg.LAYOUT_STREAMS}


@pytest.fixture(scope="module")
def lib():
    return pkg.load()


def _python_plan(table, world, F, layout, fpc, base):
    """shard.gather_frames' steps 1 and 4 on a host table [world, F]"""
    sizes = torch.from_numpy((table & 0xFFFFFFFF).astype(np.int64))
    draws = torch.from_numpy((table >> 32).astype(np.int64) & 0xFF)
    poffs = [shard.packed_offsets(sizes[r]) for r in range(world)]
    totals = [int(p[-1]) for p in poffs]
    bases = np.concatenate([[0], np.cumsum(totals)[:-1]]).astype(np.int64)
    nf = world * F
    offs = np.zeros(nf, dtype=np.int64)
    sz = np.zeros(nf, dtype=np.int64)
    dr = np.zeros(nf, dtype=np.int64)
    for r in range(world):
        fid = shard.global_frame_ids(F, r, world, layout, fpc).numpy()
        offs[fid] = bases[r] + poffs[r][:-1].numpy()
        sz[fid] = sizes[r].numpy()
        dr[fid] = draws[r].numpy()
    ids, keep = shard.assign_identifiers(torch.from_numpy(dr), base, layout, fpc)
    ids = np.where(keep.numpy(), np.uint64(0xFFFFFFFFFFFFFFFF), ids.numpy().astype(np.uint64))
    return np.array(totals, dtype=np.uint64), offs.astype(np.uint64), sz.astype(np.uint32), ids, dr


@pytest.mark.parametrize("layout", sorted(LAYOUTS))
def test_gather_plan_vs_shard(lib, layout):
    rng = np.random.default_rng(len(layout))
    for trial in range(60):
        world = int(rng.integers(1, 9))
        fpc = int(rng.choice([1, 2, 4, 16])) if layout == "streams" else 1
        F = fpc * int(rng.integers(1, 6))
        sizes = rng.integers(14, 200000, (world, F)).astype(np.uint64)
        sizes[rng.random((world, F)) < 0.1] = rng.integers(14, 40)  # small frames
        if layout == "streams":
            draws = np.zeros((world, F), dtype=np.uint64)
            draws[:, ::fpc] = 1  # each stream's primary frame draws once
            fb = rng.random((world, F)) < 0.1  # fallbacks: 3 primary, 2 secondary
            draws[fb] = np.where(draws[fb] == 1, 3, 2)
        else:
            draws = rng.choice([1, 1, 1, 3], (world, F)).astype(np.uint64)
        table = sizes | (draws << np.uint64(32))
        base = int(rng.integers(0, 1 << 40))
        rc, rb, offs, sz, ids = lib.gather_plan(table.reshape(-1), world, F, LAYOUTS[layout], fpc, base)
        assert rc == 0, (trial, api.error_name(rc))
        w_rb, w_offs, w_sz, w_ids, _ = _python_plan(table, world, F, layout, fpc, base)
        assert (rb == w_rb).all() and (offs == w_offs).all() and (sz == w_sz).all(), trial
        assert (ids == w_ids).all(), trial


def test_gather_plan_refusals(lib):
    F, world = 4, 3
    sizes = np.full((world, F), 1000, dtype=np.uint64)
    ok = sizes | (np.uint64(1) << np.uint64(32))
    # a frame with an error value: nothing to gather
    bad = ok.copy()
    bad[1, 2] = np.uint64((1 << 32) - 41) | (np.uint64(1) << np.uint64(32))  # -(DST_TOO_SMALL)
    assert api.error_name(lib.gather_plan(bad.reshape(-1), world, F, LAYOUTS["block"])[0]) == "GENERIC"
    # a frame layout whose frame made no draw (a secondary pass): refused when identifiers are asked for
    nodraw = ok.copy()
    nodraw[2, 1] = np.uint64(1000)
    assert api.error_name(lib.gather_plan(nodraw.reshape(-1), world, F, LAYOUTS["roundrobin"])[0]) == \
        "PARAMS_INVALID"
    assert lib.gather_plan(nodraw.reshape(-1), world, F, LAYOUTS["roundrobin"], want_ids=False)[0] == 0
    # streams: frames of one stream after its first draw take identifiers; no refusal
    assert lib.gather_plan(nodraw.reshape(-1), world, F, LAYOUTS["streams"], fpc=2)[0] == 0
    # layout / fpc
    assert api.error_name(lib.gather_plan(ok.reshape(-1), world, F, LAYOUTS["streams"], fpc=3)[0]) == \
        "PARAMS_INVALID"
    assert api.error_name(lib.gather_plan(ok.reshape(-1), world, F, 7)[0]) == "GENERIC"
