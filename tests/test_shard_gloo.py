"""Multi-rank path of SURVEY.md 8(e) on CPU: the frame gather to rank 0
(all_gather of sizes and identifier-draw counts, packing at 8-byte aligned
offsets that reads only the compressed bytes, batched point-to-point
receives into the root buffer, f-order table, identifiers from the scan of
the gathered draw counts, and the refusal to patch without them for
parameter sets whose draws depend on the outcomes), world size 2 over gloo."""
import socket

import pytest
import torch.multiprocessing as mp

import _shard_worker


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(*args):
    mp.spawn(_shard_worker.run, args=(2, _free_port()) + args, nprocs=2, join=True)


@pytest.mark.parametrize("layout", ["roundrobin", "block"])
def test_gather_world2(orc, layout):
    _spawn(5, 3000, layout, "ok")


def test_gather_world2_ragged_small(orc):
    # frames shorter than the GPU segment, odd sizes (byte-granular compaction)
    _spawn(7, 17, "roundrobin", "ok")


def test_gather_world2_error_value(orc):
    _spawn(3, 500, "roundrobin", "error")


def test_gather_world2_patch_refused_with_secondary_passes(orc):
    _spawn(3, 500, "roundrobin", "patch_refused")


@pytest.mark.parametrize("layout", ["roundrobin", "block"])
def test_gather_world2_patch_refused_with_draws_and_secondary_passes(orc, layout):
    """per-frame draw counts do not make a frame layout with
    secondary passes patchable (a secondary frame followed its rank's previous
    frame); refused with and without the parameters at hand."""
    _spawn(3, 500, layout, "patch_refused_draws")


@pytest.mark.parametrize("layout", ["roundrobin", "block"])
def test_gather_world2_patch_refused_on_one_rank_only(orc, layout):
    """Only one rank's draw counts hold a 0 (a secondary pass): the refusal is
    collective, every rank raises before the gather."""
    _spawn(3, 500, layout, "patch_refused_one_rank")


def test_gather_world2_fallback_identifiers_vs_one_context(orc):
    """Round-robin frames with the uncompressed fallback (three draws per
    fallback frame): after the gather every frame, identifier included, equals
    ONE context's call loop over all frames in global order."""
    _spawn(8, 700, "roundrobin", "fallback")


def test_gather_world2_streams_model_vs_call_loop(orc):
    """Streams of 5 frames (MODEL secondary passes, fallback enabled) sharded
    s mod 2: every gathered frame, identifier included, equals one process's
    c-major call loop over all the streams' contexts."""
    _spawn(10, 600, "streams", "streams")
