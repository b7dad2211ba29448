"""Multi-rank path of SURVEY.md 8(e) on CPU: the frame gather to rank 0
(all_gather of sizes, packing at 8-byte aligned offsets that reads only the
compressed bytes, batched point-to-point receives into the root buffer,
f-order table, identifier patch and its refusal for parameter sets whose
identifiers depend on the outcomes), world size 2 over gloo."""
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
