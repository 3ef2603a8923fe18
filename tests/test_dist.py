"""Multi-rank host logic of the sharded path on CPU (gloo, world_size 2).

The GPU path shards packets by contiguous range and exchanges one summary per
flow (fluere_amd/dist.py); the device merge itself is covered on the GPU by
test_gpu_parity.py::test_sharded_merge_equals_single.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fluere_amd import dist as fdist
from fluere_amd._lib import SUMMARY_BYTES, SUMMARY_DTYPE


@pytest.mark.parametrize("n", [0, 1, 2, 3, 7, 1000, 10_000_001])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    got = [fdist.shard_range(n, r, world) for r in range(world)]
    pos = 0
    for first, cnt in got:
        assert cnt >= 0
        if cnt:
            assert first == pos
        pos += cnt
    assert pos == n
    sizes = [c for _, c in got if c]
    if sizes:
        assert max(sizes) - min(sizes) <= max(1, (n + world - 1) // world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _summaries(rank, n):
    a = np.zeros(n, dtype=SUMMARY_DTYPE)
    a["key"][:, 0] = rank * 1000 + np.arange(n)
    a["pkts"][:, 0] = np.arange(n) + 1
    a["last"] = (rank << 32) + np.arange(n)
    return torch.from_numpy(a.view(np.uint8).copy())


def _worker(rank, world, port, counts, tmins, tmaxs, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = _summaries(rank, counts[rank])
        got = fdist.gather_summaries(s, tmins[rank], tmaxs[rank], dst=0)
        if rank == 0:
            allsum, gmin, gmax = got
            q.put((allsum.numpy().tobytes(), gmin, gmax))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("counts,tmins,tmaxs", [
    ([3, 5], [100, 50], [200, 400]),
    ([4, 0], [10, fdist.NONE64], [20, 0]),      # an empty shard
    ([0, 0], [fdist.NONE64, fdist.NONE64], [0, 0]),
])
def test_gather_summaries_gloo(counts, tmins, tmaxs):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, tmins, tmaxs, q)) for r in range(world)]
    for p in procs:
        p.start()
    raw, gmin, gmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = b"".join(_summaries(r, counts[r]).numpy().tobytes() for r in range(world))
    assert raw == want and len(raw) == sum(counts) * SUMMARY_BYTES
    lows = [t for t in tmins if t != fdist.NONE64]
    assert gmin == (min(lows) if lows else fdist.NONE64)
    assert gmax == max(tmaxs)
