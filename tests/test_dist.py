"""Multi-rank host logic of the sharded path on CPU (gloo, world_size 2 and 3).

The GPU path shards packets by contiguous range; every rank exports one block
per owner rank and one all-to-all delivers them (fluere_amd/dist.py).  The
device export / merge / composition is covered on the GPU by
test_gpu_parity.py (logical shards on one device, and a 2-rank gloo run of
ShardExchange itself).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fluere_amd import dist as fdist


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


def _worker(rank, world, port, blk, q):
    """One rank of the exchange: block o of every rank's send buffer carries
    (rank, o) in its bytes; after the all-to-all, rank o's receive buffer
    must hold the blocks for o from ranks 0..world-1, in rank order.  Also the
    capacity agreement (largest per-owner counts over all ranks)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        send = torch.zeros(world * blk, dtype=torch.uint8)
        for o in range(world):
            send[o * blk:(o + 1) * blk] = torch.arange(blk, dtype=torch.int64).to(torch.uint8) ^ (16 * rank + o)
        recv = torch.empty_like(send)
        fdist.exchange_blocks(send, recv)
        need = fdist.agree_need(100 * rank + 7, 3 - rank)
        q.put((rank, recv.numpy().tobytes(), need))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,blk", [(2, 64), (2, 4096), (3, 256)])
def test_exchange_blocks_gloo(world, blk):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, blk, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (raw, need)) for r, raw, need in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    base = np.arange(blk, dtype=np.int64).astype(np.uint8)
    for o in range(world):
        raw, need = got[o]
        want = b"".join((base ^ (16 * r + o)).tobytes() for r in range(world))
        assert raw == want, f"owner {o}: blocks out of place"
        assert need == (100 * (world - 1) + 7, 3)


def test_order_records_merges_ranks():
    from fluere_amd._lib import RECORD_DTYPE
    a = np.zeros(3, dtype=RECORD_DTYPE)
    b = np.zeros(2, dtype=RECORD_DTYPE)
    a["order_key"] = [40, fdist.NONE64, 7]
    a["first"] = [1, 5, 2]
    b["order_key"] = [fdist.NONE64, 12]
    b["first"] = [3, 4]
    recs, ne = fdist.order_records([a, b])
    assert ne == 3
    assert list(recs["order_key"][:3]) == [7, 12, 40]
    assert list(recs["first"][3:]) == [3, 5]


def _var_worker(rank, world, port, q):
    """exchange_var: rank r sends (r + 1) * (o + 1) records of 3 bytes to rank
    o, each byte = 16 * r + o; every rank receives its segments in rank order
    with the right counts.  Also the communicator's all-gather and MAX."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts = np.array([(rank + 1) * (o + 1) for o in range(world)], dtype=np.uint64)
        send = torch.cat([torch.full((int(c) * 3,), 16 * rank + o, dtype=torch.uint8) for o, c in enumerate(counts)])
        recv, rc = fdist.exchange_var(send, counts, 3)
        n = int(rc.sum()) * 3
        comm = fdist._DistComm.__new__(fdist._DistComm)
        comm.group, comm.world, comm.ranks, comm.gloo = None, world, [rank], True
        comm.device = torch.device("cpu")
        comm.same_stream = True
        g = comm.allgather([np.array([rank, 10 * rank], dtype=np.int64)])
        m = comm.allreduce_max([np.array([rank, -rank], dtype=np.int64)])
        # the wire path: sizes every rank knows from one gather of a vector
        gd = comm.allgather_dev([torch.tensor([rank, 7] + [int(c) * 3 for c in counts], dtype=torch.int64)])
        sizes = gd[:, 2:]
        (rk,) = comm.all_to_all_known([send], [sizes[rank]], [sizes[:, rank]])
        q.put((rank, recv[:n].numpy().tobytes(), [int(x) for x in rc], g.tolist(), m.tolist(), gd.tolist(),
               rk[:int(sizes[:, rank].sum())].numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_var_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_var_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for o in range(world):
        raw, rc, g, m, gd, rk = got[o]
        assert rc == [(r + 1) * (o + 1) for r in range(world)]
        want = b"".join(bytes([16 * r + o]) * (3 * (r + 1) * (o + 1)) for r in range(world))
        assert raw == want
        assert rk == want  # exchange_known with the gathered sizes moves the same bytes
        assert g == [[r, 10 * r] for r in range(world)]
        assert m == [world - 1, 0]
        assert gd == [[r, 7] + [3 * (r + 1) * (x + 1) for x in range(world)] for r in range(world)]



def test_order_records_sweep_words():
    """Sharded sweep records: ties of the ending packet's index are broken by
    the order words (FIN/RST close first, then by exp, then by the firing
    entry's creation), not by `first`."""
    from fluere_amd._lib import RECORD_DTYPE
    a = np.zeros(3, dtype=RECORD_DTYPE)
    b = np.zeros(2, dtype=RECORD_DTYPE)
    a["order_key"] = [50, 50, fdist.NONE64]
    a["first"] = [1, 2, 3]
    b["order_key"] = [50, 20]
    b["first"] = [0, 9]
    aa = np.array([[101, 7], [101, 3], [0, 0]], dtype=np.uint64)
    ab = np.array([[0, 0], [0, 0]], dtype=np.uint64)
    recs, ne = fdist.order_records([a, b], [aa, ab])
    assert ne == 4
    assert list(recs["order_key"]) == [20, 50, 50, 50, fdist.NONE64]
    assert list(recs["first"]) == [9, 0, 2, 1, 3]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_bench_c4_is_the_fixed_100m_capture(world):
    """bench.py --config c4 is BASELINE configs[3] as named --
    100M IMIX packets sharded over N GPUs (strong scaling), every packet in
    exactly one rank's shard; c4_shard keeps the 12.5M-per-GPU shard (weak)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from fluere_amd import dist as fdist
    C = bench.CONFIGS["c4"]
    n = bench.packets_total(C, world)
    assert n == 100_000_000
    assert sum(fdist.shard_range(n, r, world)[1] for r in range(world)) == n
    assert bench.packets_total(bench.CONFIGS["c4_shard"], world) == 12_500_000 * world
