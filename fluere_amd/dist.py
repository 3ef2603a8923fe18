"""Packet-range sharding over GPUs: one process per GPU (torch.distributed,
backend "nccl" = RCCL on ROCm).  The one exchange is the flow-table merge:
every rank exports its flows into one block per owner rank (owner = hash of
the canonical key), one all-to-all over xGMI delivers them, and every owner
merges and finalizes its own flows (fluere_export_device /
fluere_merge_gathered in include/fluere_gpu.h).

Reference: the offline loop is one sequential pass (offline_fluereflows.rs:68-176).
Shard r processes packets [r*N/G, (r+1)*N/G) with global packet indices, so
order-free record fields merge as sums / min / max, and the flows whose record
depends on packet order are composed at their owner from per-shard pieces of
the state machine (the annex of fluere_gpu.h).

When the capture's span reaches the timeout, the hard-timeout sweep
(offline_fluereflows.rs:103-119,161-175) couples the shards: an expiry entry
fires at the first processed packet of the whole capture with t >= exp.  The
merge is then completed by the sweep composition (_sweep_compose): the shards
ship their packets' metadata to the keys' owners, compute the sweep points over
their own packets (asking later shards for the rest), and the owners run the
exact chase until the processed-packet set is stable (fluere_sweep_* in
include/fluere_gpu.h).

The protocol is written once (_shard_step) over a small communicator: _DistComm
(torch.distributed, one context per process) for ShardExchange, _LocalComm
(device copies, G contexts in one process) for LogicalShards -- the latter is
SURVEY.md section 8e's "testing without 8 GPUs" and runs the same calls.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import RECORD_DTYPE, Stats, check

NONE64 = (1 << 64) - 1
SPAN_BIAS = 1 << 62  # fluere_export_async d_info[4] = SPAN_BIAS - earliest valid time
# wide blocks of at least this many bytes travel in the compact wire encoding
# (fluere_wire_pack / fluere_wire_unpack): variable-length summaries, split
# sizes exact per owner; smaller ones go as equal wide blocks (one fewer pass)
WIRE_MIN_BLOCK = 1 << 20
WIRE_SLOT_PREFIX = 16       # fluere_wire_pack_slots: the size word before each slot's block
WIRE_SLOT_HEADROOM = 1 / 16  # slot = largest block of the last host-driven step + this share


def shard_range(n_packets: int, rank: int, world: int):
    per = (n_packets + world - 1) // world
    first = min(n_packets, rank * per)
    return first, min(n_packets, first + per) - first


def set_index_base(ctx, base: int):
    check(_lib.lib().fluere_set_index_base(ctx._h, base), "fluere_set_index_base")
    ctx.index_base = int(base)


def _pow2_at_least(n: int, lo: int) -> int:
    c = max(1, lo)
    while c < n:
        c *= 2
    return c


def agree_need(need: int, need_annex: int, group=None, device=None):
    """Largest per-owner counts over all ranks (every rank must size the
    blocks alike): one small all-reduce."""
    import torch
    import torch.distributed as dist
    gloo = dist.get_backend(group) == "gloo"
    t = torch.tensor([need, need_annex], dtype=torch.int64, device="cpu" if gloo else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    a, b = t.tolist()
    return int(a), int(b)


def exchange_blocks(send, recv, group=None):
    """All-to-all of equal blocks: block o of rank r's `send` lands at block r
    of rank o's `recv` (RCCL over xGMI; gloo moves host copies)."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        s_h, r_h = send.cpu(), torch.empty(recv.numel(), dtype=recv.dtype)
        dist.all_to_all_single(r_h, s_h, group=group)
        recv.copy_(r_h)
    else:
        dist.all_to_all_single(recv, send, group=group)


def exchange_known(send, send_counts, recv_counts, group=None):
    """All-to-all of byte runs whose sizes every rank already knows (the
    gathered wire sizes): send_counts[o] bytes for rank o, recv_counts[s]
    bytes from rank s, both in rank order.  Returns the received bytes."""
    import torch
    import torch.distributed as dist
    ins = [int(x) for x in send_counts]
    outs = [int(x) for x in recv_counts]
    n_out = sum(outs)
    recv = torch.empty(max(1, n_out), dtype=torch.uint8, device=send.device)
    if dist.get_backend(group) == "gloo":
        s_h = send[: sum(ins)].cpu() if send.is_cuda else send[: sum(ins)]
        r_h = torch.empty(n_out, dtype=torch.uint8)
        dist.all_to_all_single(r_h, s_h, outs, ins, group=group)
        recv[:n_out].copy_(r_h)
    else:
        dist.all_to_all_single(recv[:n_out], send[: sum(ins)], outs, ins, group=group)
    return recv


def exchange_var(send, send_counts, elem: int, group=None):
    """All-to-all with per-destination sizes: send holds send_counts[o]
    elements of `elem` bytes for rank o, in rank order.  Returns (recv,
    recv_counts): recv_counts[s] elements from rank s, in rank order."""
    import torch
    import torch.distributed as dist
    gloo = dist.get_backend(group) == "gloo"
    world = dist.get_world_size(group)
    dev = "cpu" if gloo else send.device
    sc = torch.tensor(np.asarray(send_counts, dtype=np.int64), dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = np.asarray(rc.tolist(), dtype=np.uint64)
    n_out = int(recv_counts.sum()) * elem
    ins = [int(x) * elem for x in send_counts]
    outs = [int(x) * elem for x in recv_counts]
    if gloo:
        s_h = send[: sum(ins)].cpu() if send.is_cuda else send[: sum(ins)]
        r_h = torch.empty(n_out, dtype=torch.uint8)
        dist.all_to_all_single(r_h, s_h, outs, ins, group=group)
        recv = torch.empty(max(1, n_out), dtype=torch.uint8, device=send.device)
        recv[:n_out].copy_(r_h)
    else:
        recv = torch.empty(max(1, n_out), dtype=torch.uint8, device=send.device)
        dist.all_to_all_single(recv[:n_out], send[: sum(ins)], outs, ins, group=group)
    return recv, recv_counts


class _DistComm:
    """This process's one context over torch.distributed.  With RCCL the
    collectives run on torch's current stream; a context on a stream of its
    own is synchronised around them (the library's calls that feed a
    collective end with their stream drained, and a collective's output is
    waited for before the library reads it)."""

    host_reads = 0  # values read back to the host (each one a round trip)

    def __init__(self, group, ctx):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.ranks = [dist.get_rank(group)]
        self.gloo = dist.get_backend(group) == "gloo"
        self.device = torch.device("cuda", torch.cuda.current_device())
        cur = torch.cuda.current_stream().cuda_stream
        self.same_stream = ctx.stream is not None and int(ctx.stream) != 0 and int(ctx.stream) == int(cur)

    def _before(self):
        import torch
        if not self.same_stream:
            torch.cuda.synchronize()  # the context's kernels (any stream) before the collective

    def _after(self):
        import torch
        if not self.same_stream and not self.gloo:
            torch.cuda.current_stream().synchronize()  # the collective before the context reads its output

    def allreduce_max_dev(self, tensors):
        import torch.distributed as dist
        (t,) = tensors
        self._before()
        x = t.cpu() if self.gloo else t
        dist.all_reduce(x, op=dist.ReduceOp.MAX, group=self.group)
        self._after()
        self.host_reads += 1
        return np.asarray(x.tolist(), dtype=np.int64)

    def allgather_dev(self, tensors):
        """Every rank's device vector -> (world, k) on the host (one read)."""
        import torch
        import torch.distributed as dist
        (t,) = tensors
        self._before()
        x = t.cpu() if self.gloo else t
        out = torch.empty((self.world, x.numel()), dtype=x.dtype, device=x.device)
        if self.gloo:
            dist.all_gather(list(out.unbind(0)), x, group=self.group)
        else:
            dist.all_gather_into_tensor(out, x, group=self.group)
        self._after()
        self.host_reads += 1
        return np.asarray(out.tolist(), dtype=np.int64)

    def all_to_all_known(self, sends, send_counts, recv_counts):
        (s,), (sc,), (rc,) = sends, send_counts, recv_counts
        self._before()
        r = exchange_known(s, sc, rc, self.group)
        self._after()
        return [r]

    def allreduce_max(self, arrays):
        import torch
        import torch.distributed as dist
        (a,) = arrays
        t = torch.tensor(np.asarray(a, dtype=np.int64), device="cpu" if self.gloo else self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        self.host_reads += 1
        return np.asarray(t.tolist(), dtype=np.int64)

    def allgather(self, arrays):
        import torch
        import torch.distributed as dist
        (a,) = arrays
        a = np.asarray(a, dtype=np.int64)
        t = torch.tensor(a, device="cpu" if self.gloo else self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        self.host_reads += 1
        return np.stack([np.asarray(o.tolist(), dtype=np.int64) for o in out])

    def all_to_all_equal(self, sends, recvs):
        (s,), (r,) = sends, recvs
        self._before()
        exchange_blocks(s, r, self.group)
        self._after()

    def all_to_all_v(self, sends, counts, elem):
        (s,), (c,) = sends, counts
        self._before()
        self.host_reads += 1  # (the receive counts)
        r, rc = exchange_var(s, c, elem, self.group)
        self._after()
        return [r], [rc]


class _LocalComm:
    """G contexts of one process (logical shards on one device): every
    collective is a set of device copies."""

    def __init__(self, n):
        self.world = n
        self.ranks = list(range(n))
        self.host_reads = 0

    @staticmethod
    def _sync():
        import torch
        torch.cuda.synchronize()  # (the contexts run on streams of their own)

    def allreduce_max_dev(self, tensors):
        self._sync()
        self.host_reads += 1
        return np.max(np.stack([np.asarray(t.tolist(), dtype=np.int64) for t in tensors]), axis=0)

    def allgather_dev(self, tensors):
        self._sync()
        self.host_reads += 1
        return np.stack([np.asarray(t.tolist(), dtype=np.int64) for t in tensors])

    def all_to_all_known(self, sends, send_counts, recv_counts):
        recvs, _ = self.all_to_all_v(sends, send_counts, 1)
        return recvs

    def allreduce_max(self, arrays):
        return np.max(np.stack([np.asarray(a, dtype=np.int64) for a in arrays]), axis=0)

    def allgather(self, arrays):
        return np.stack([np.asarray(a, dtype=np.int64) for a in arrays])

    def all_to_all_equal(self, sends, recvs):
        self._sync()
        G = self.world
        blk = sends[0].numel() // G
        for o in range(G):
            for r in range(G):
                recvs[o][r * blk:(r + 1) * blk].copy_(sends[r][o * blk:(o + 1) * blk])
        self._sync()

    def all_to_all_v(self, sends, counts, elem):
        import torch
        self._sync()
        G = self.world
        offs = [np.concatenate([[0], np.cumsum(np.asarray(c, dtype=np.uint64))]).astype(np.int64) for c in counts]
        recvs, rcounts = [], []
        for o in range(G):
            parts = [sends[r][int(offs[r][o]) * elem:int(offs[r][o + 1]) * elem] for r in range(G)]
            n = sum(p.numel() for p in parts)
            out = torch.empty(max(1, n), dtype=torch.uint8, device="cuda")
            if n:
                torch.cat(parts, out=out[:n])
            recvs.append(out)
            rcounts.append(np.asarray([counts[r][o] for r in range(G)], dtype=np.uint64))
        self._sync()
        return recvs, rcounts


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _buf(nbytes: int):
    import torch
    return torch.empty(max(1, int(nbytes)), dtype=torch.uint8, device="cuda")


def _arr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _sweep_pack(comm, ctxs):
    """Step 1 of the sweep composition, run after the export and before the
    owner merge (which replaces the context's flow table with its owner's):
    every shard's valid packets as 32-byte records per owner rank."""
    L = _lib.lib()
    W = comm.world
    counts, sends = [], []
    for c in ctxs:
        cnt = np.zeros(W, np.uint64)
        check(L.fluere_sweep_pack(c._h, W, _arr(cnt), None), "fluere_sweep_pack")
        b = _buf(int(cnt.sum()) * 32)
        check(L.fluere_sweep_pack(c._h, W, _arr(cnt), b.data_ptr()), "fluere_sweep_pack")
        counts.append(cnt)
        sends.append(b)
    return counts, sends


def _sweep_compose(comm, ctxs, rank_first, counts, sends):
    """The hard-timeout sweep across shards (include/fluere_gpu.h,
    fluere_sweep_*): every local context is a holder (its packet range) and an
    owner (its flows).  rank_first: first global packet index of every rank,
    plus the total (world + 1 entries); counts / sends: _sweep_pack's."""
    L = _lib.lib()
    W = comm.world
    u64 = np.uint64
    # 1-2. packets to their keys' owners
    recvs, rcounts = comm.all_to_all_v(sends, counts, 32)
    for c, r, rc in zip(ctxs, recvs, rcounts):
        rc = np.ascontiguousarray(rc, dtype=u64)
        check(L.fluere_sweep_load(c._h, r.data_ptr(), W, _arr(rc)), "fluere_sweep_load")
    del sends, recvs
    # 3. the processed-packet fixed point
    back = [None] * len(ctxs)
    passes = 0
    while True:
        passes += 1
        mts = []
        for c, b in zip(ctxs, back):
            m = ctypes.c_uint64()
            check(L.fluere_sweep_index(c._h, _ptr(b), ctypes.byref(m)), "fluere_sweep_index")
            mts.append(np.array([m.value & ((1 << 63) - 1)], dtype=np.int64))
        allmax = np.ascontiguousarray(comm.allgather(mts).reshape(W).astype(u64))
        qsends, qcounts = [], []
        for c, rk in zip(ctxs, comm.ranks):
            qc = np.zeros(W, u64)
            check(L.fluere_sweep_queries(c._h, W, rk, _arr(allmax), _arr(qc), None), "fluere_sweep_queries")
            b = _buf(int(qc.sum()) * 8)
            tmp = np.zeros(W, u64)
            check(L.fluere_sweep_queries(c._h, W, rk, _arr(allmax), _arr(tmp), b.data_ptr()), "fluere_sweep_queries")
            qsends.append(b)
            qcounts.append(qc)
        qrecv, qrc = comm.all_to_all_v(qsends, qcounts, 8)
        asends = []
        for c, q, n in zip(ctxs, qrecv, qrc):
            n = int(np.asarray(n, dtype=u64).sum())
            a = _buf(n * 8)
            check(L.fluere_sweep_answer(c._h, q.data_ptr(), n, a.data_ptr()), "fluere_sweep_answer")
            asends.append(a)
        arecv, _ = comm.all_to_all_v(asends, qrc, 8)
        fsends = []
        for c, a, cnt in zip(ctxs, arecv, counts):
            f = _buf(int(cnt.sum()) * 8)
            check(L.fluere_sweep_points(c._h, a.data_ptr(), f.data_ptr()), "fluere_sweep_points")
            fsends.append(f)
        frecv, _ = comm.all_to_all_v(fsends, counts, 8)
        prs, chg = [], []
        for c, f, rc in zip(ctxs, frecv, rcounts):
            p = _buf(int(np.asarray(rc, dtype=u64).sum()))
            ch = ctypes.c_int()
            check(L.fluere_sweep_chase(c._h, f.data_ptr(), p.data_ptr(), ctypes.byref(ch)), "fluere_sweep_chase")
            prs.append(p)
            chg.append(np.array([ch.value], dtype=np.int64))
        if not int(comm.allreduce_max(chg)[0]):
            break
        back, _ = comm.all_to_all_v(prs, rcounts, 1)
    # 4. seeds of the creating packets from their holders
    rf = np.ascontiguousarray(np.asarray(rank_first, dtype=u64))
    reqs, scounts = [], []
    for c in ctxs:
        sc = np.zeros(W, u64)
        check(L.fluere_sweep_seed_requests(c._h, W, _arr(rf), _arr(sc), None), "fluere_sweep_seed_requests")
        b = _buf(int(sc.sum()) * 8)
        check(L.fluere_sweep_seed_requests(c._h, W, _arr(rf), _arr(sc), b.data_ptr()), "fluere_sweep_seed_requests")
        reqs.append(b)
        scounts.append(sc)
    rrecv, rrc = comm.all_to_all_v(reqs, scounts, 8)
    ssends = []
    for c, q, n in zip(ctxs, rrecv, rrc):
        n = int(np.asarray(n, dtype=u64).sum())
        b = _buf(n * 40)
        check(L.fluere_sweep_seeds(c._h, q.data_ptr(), n, b.data_ptr()), "fluere_sweep_seeds")
        ssends.append(b)
    srecv, _ = comm.all_to_all_v(ssends, rrc, 40)
    # 5. records
    stats = []
    for c, sd in zip(ctxs, srecv):
        st = Stats()
        check(L.fluere_sweep_finish(c._h, sd.data_ptr(), ctypes.byref(st)), "fluere_sweep_finish")
        d = st.as_dict()
        d["sweep_passes"] = passes
        stats.append(d)
    return stats


class _StepState:
    def __init__(self, cap, cap_annex, wire=None):
        self.cap, self.cap_annex = max(1, int(cap)), max(1, int(cap_annex))
        self.sends = self.recvs = None
        self.blk = 0
        self.infos = None
        self.wsends = None
        self.wbound = 0
        self.wire = wire  # None: by block size (WIRE_MIN_BLOCK); True / False: always / never
        self.bytes_sent = 0  # per local context, last step: the bytes it sent to other ranks
        self.wire_used = False
        # the device-agreed step (_shard_step_dev): taken after a host-driven
        # step that needed neither annexes nor the sweep composition
        self.dev_next = False
        self.flags = None
        self.device_agreed = False  # the last step was the device-agreed one
        # the device-agreed step's wire slots (fluere_wire_pack_slots): bytes
        # per owner, sized from the last host-driven wire step's largest block
        # (+ WIRE_SLOT_HEADROOM); 0 until a host-driven step used the wire
        self.wslot = 0
        self.wslot_sends = self.wslot_recvs = None


def _ensure_blocks(S: _StepState, n_ctx: int, W: int, blk: int):
    import torch
    if S.sends is None or S.blk != blk or len(S.sends) != n_ctx:
        S.sends = [torch.empty(W * blk, dtype=torch.uint8, device="cuda") for _ in range(n_ctx)]
        S.recvs = [torch.empty(W * blk, dtype=torch.uint8, device="cuda") for _ in range(n_ctx)]
        S.blk = blk


def _shard_step_dev(comm, ctxs, S: _StepState):
    """The step agreed on the device: parse + key + aggregate, export without
    annexes into blocks of the current capacities, one all-to-all of equal
    blocks, the owner merge -- enqueued back to back on the stream.  Each
    merge sets a retry word on the device (a block cut short, order-dependent
    flows, the span reaching the timeout); the ranks reduce it (MAX) and read
    it once: the step's one host round trip.  Returns the stats, or None when
    the step must be redone by the host-driven sequence."""
    import torch
    L = _lib.lib()
    W = comm.world
    for c in ctxs:
        c.parse_aggregate()
    blk = int(L.fluere_shard_block_bytes(S.cap, S.cap_annex))
    _ensure_blocks(S, len(ctxs), W, blk)
    if S.infos is None or len(S.infos) != len(ctxs) or S.infos[0].numel() < 6:
        S.infos = [torch.zeros(6, dtype=torch.int64, device="cuda") for _ in ctxs]
    if S.flags is None or len(S.flags) != len(ctxs):
        S.flags = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in ctxs]
    # the compact wire encoding in fixed slots when the blocks are large (the
    # host-driven step's rule), sized by the last host-driven wire step
    wire = (blk >= WIRE_MIN_BLOCK) if S.wire is None else bool(S.wire)
    slot = S.wslot if wire else 0
    for c, rk, s, info in zip(ctxs, comm.ranks, S.sends, S.infos):
        check(L.fluere_export_async(c._h, s.data_ptr(), W, rk, S.cap, S.cap_annex, info.data_ptr()),
              "fluere_export_async")
    if slot:
        if S.wslot_sends is None or S.wslot_sends[0].numel() != W * slot or len(S.wslot_sends) != len(ctxs):
            S.wslot_sends = [torch.empty(W * slot, dtype=torch.uint8, device="cuda") for _ in ctxs]
            S.wslot_recvs = [torch.empty(W * slot, dtype=torch.uint8, device="cuda") for _ in ctxs]
        for c, s, ws in zip(ctxs, S.sends, S.wslot_sends):
            check(L.fluere_wire_pack_slots(c._h, s.data_ptr(), W, S.cap, S.cap_annex, slot, ws.data_ptr()),
                  "fluere_wire_pack_slots")
        comm.all_to_all_equal(S.wslot_sends, S.wslot_recvs)
        for c, wr, r in zip(ctxs, S.wslot_recvs, S.recvs):
            check(L.fluere_wire_unpack_slots(c._h, wr.data_ptr(), W, slot, S.cap, S.cap_annex, r.data_ptr()),
                  "fluere_wire_unpack_slots")
    else:
        comm.all_to_all_equal(S.sends, S.recvs)
    for c, r, f in zip(ctxs, S.recvs, S.flags):
        check(L.fluere_merge_gathered_async(c._h, r.data_ptr(), W, S.cap, S.cap_annex, f.data_ptr()),
              "fluere_merge_gathered_async")
    redo = int(comm.allreduce_max_dev(S.flags)[0])
    stats = []
    for c in ctxs:
        st = Stats()
        rc = L.fluere_merge_gathered_finish(c._h, ctypes.byref(st))
        if rc == _lib.RETRY and redo:
            continue
        check(rc, "fluere_merge_gathered_finish")
        d = st.as_dict()
        d["rc"] = rc
        d["device_agreed"] = 1
        stats.append(d)
    if redo:
        return None
    S.wire_used = bool(slot)
    S.bytes_sent = (W - 1) * (slot if slot else blk)
    return stats


def _shard_step(comm, ctxs, S: _StepState, rank_first_fn):
    """One sharded pass over every local context: the device-agreed step
    when the last step allows it (_shard_step_dev), else -- or when it asks
    for a redo -- the host-driven one."""
    blk = int(_lib.lib().fluere_shard_block_bytes(S.cap, S.cap_annex))
    wire = (blk >= WIRE_MIN_BLOCK) if S.wire is None else bool(S.wire)
    if S.dev_next and (not wire or S.wslot):
        stats = _shard_step_dev(comm, ctxs, S)
        if stats is not None:
            S.device_agreed = True
            return stats
    S.device_agreed = False
    return _shard_step_host(comm, ctxs, S, rank_first_fn)


def _shard_step_host(comm, ctxs, S: _StepState, rank_first_fn):
    """One sharded pass over every local context (parse + key + aggregate,
    export, capacity agreement, all-to-all, owner merge; the sweep
    composition when the span reaches the timeout), every decision taken on
    the host from the gathered export counts.  Returns the merge stats of
    every local context."""
    import torch
    L = _lib.lib()
    W = comm.world
    for c in ctxs:
        c.parse_aggregate()
    annexes = expiry = False
    timeout_us = int(ctxs[0].timeout_ms) * 1000
    sizes = None  # wire: (world, W) bytes of every rank's block for every owner
    while True:
        blk = int(L.fluere_shard_block_bytes(S.cap, S.cap_annex))
        wire = (blk >= WIRE_MIN_BLOCK) if S.wire is None else bool(S.wire)  # (the same on every rank)
        _ensure_blocks(S, len(ctxs), W, blk)
        if wire:
            wb = int(L.fluere_wire_bound(S.cap, S.cap_annex))
            if S.wsends is None or S.wbound != wb or len(S.wsends) != len(ctxs):
                S.wsends = [torch.empty(W * wb, dtype=torch.uint8, device="cuda") for _ in ctxs]
                S.wbound = wb
        nk = 6 + (W if wire else 0)
        if S.infos is None or len(S.infos) != len(ctxs) or S.infos[0].numel() != nk:
            S.infos = [torch.zeros(nk, dtype=torch.int64, device="cuda") for _ in ctxs]
        if not annexes:
            for c, rk, s, info, ws in zip(ctxs, comm.ranks, S.sends, S.infos, S.wsends if wire else S.sends):
                check(L.fluere_export_async(c._h, s.data_ptr(), W, rk, S.cap, S.cap_annex, info.data_ptr()),
                      "fluere_export_async")
                if wire:  # the wire sizes ride in the same gathered vector
                    check(L.fluere_wire_pack(c._h, s.data_ptr(), W, S.cap, S.cap_annex, ws.data_ptr(),
                                             info.data_ptr() + 48), "fluere_wire_pack")
            g = comm.allgather_dev(S.infos)
            n0, n1, n_cplx = (int(x) for x in g[:, :3].max(axis=0))
            span0, span1 = int(g[:, 4].max()), int(g[:, 5].max())
            sizes = g[:, 6:6 + W] if wire else None
            expiry = span0 > 0 and span1 - (SPAN_BIAS - span0) >= timeout_us
            if n_cplx and not expiry:
                annexes = True  # some rank has order-dependent flows: export with annexes
                continue
        else:
            n0 = n1 = 0
            needs = []
            for c, rk, s in zip(ctxs, comm.ranks, S.sends):
                need, need_a = ctypes.c_uint64(), ctypes.c_uint64()
                check(L.fluere_export_device(c._h, s.data_ptr(), W, rk, S.cap, S.cap_annex, ctypes.byref(need),
                                             ctypes.byref(need_a)), "fluere_export_device")
                needs.append(np.array([need.value, need_a.value], dtype=np.int64))
            n0, n1 = (int(x) for x in comm.allreduce_max(needs))
            if wire and n0 <= S.cap and n1 <= S.cap_annex:
                for c, s, ws, info in zip(ctxs, S.sends, S.wsends, S.infos):
                    check(L.fluere_wire_pack(c._h, s.data_ptr(), W, S.cap, S.cap_annex, ws.data_ptr(),
                                             info.data_ptr() + 48), "fluere_wire_pack")
                sizes = comm.allgather_dev(S.infos)[:, 6:6 + W]
        if n0 <= S.cap and n1 <= S.cap_annex:
            break
        # a shard had more flows for some owner: grow the blocks, export again
        S.cap = _pow2_at_least(n0, S.cap)
        S.cap_annex = _pow2_at_least(n1, S.cap_annex)
    packed = _sweep_pack(comm, ctxs) if expiry else None
    S.wire_used = wire
    if wire:
        sizes = np.asarray(sizes, dtype=np.int64)  # sizes[r][o]: rank r's block for owner o
        rks = comm.ranks
        wrecv = comm.all_to_all_known(S.wsends, [sizes[rk] for rk in rks], [sizes[:, rk] for rk in rks])
        for c, rk, wr, r in zip(ctxs, rks, wrecv, S.recvs):
            rs = np.ascontiguousarray(sizes[:, rk].astype(np.uint64))
            check(L.fluere_wire_unpack(c._h, wr.data_ptr(), W, _arr(rs), S.cap, S.cap_annex, r.data_ptr()),
                  "fluere_wire_unpack")
        S.bytes_sent = int(sizes[rks[0]].sum() - sizes[rks[0], rks[0]])
        # the next device-agreed step's fixed slots: this step's largest block + headroom
        big = int(sizes.max()) + WIRE_SLOT_PREFIX
        S.wslot = (big + int(big * WIRE_SLOT_HEADROOM) + 255) // 256 * 256
    else:
        S.bytes_sent = (W - 1) * blk
        comm.all_to_all_equal(S.sends, S.recvs)
    stats, rcs = [], []
    for c, r in zip(ctxs, S.recvs):
        st = Stats()
        rc = L.fluere_merge_gathered(c._h, r.data_ptr(), W, S.cap, S.cap_annex, ctypes.byref(st))
        if rc not in (_lib.OK, _lib.NEED_SWEEP):
            check(rc, "fluere_merge_gathered")
        rcs.append(rc)
        d = st.as_dict()
        d["rc"] = rc
        stats.append(d)
    if any(rc == _lib.NEED_SWEEP for rc in rcs):
        if not expiry or not all(rc == _lib.NEED_SWEEP for rc in rcs):
            raise _lib.FluereError(_lib.E_STATE, "sharded merge: ranks disagree on the capture span")
        stats = _sweep_compose(comm, ctxs, rank_first_fn(), *packed)
        for d in stats:
            d["rc"] = _lib.NEED_SWEEP
    # the next step agrees on the device unless this one needed annexes or the
    # sweep (the capacities it grew to stay)
    S.dev_next = not annexes and not expiry
    return stats


class ShardExchange:
    """The multi-GPU step: parse + key + aggregate over this rank's shard,
    export into per-owner blocks (summaries of every flow, annexes of the flows
    whose record depends on packet order in this shard, whose records that
    open and close inside the shard stay here), agree on the block capacities,
    one all-to-all, owner merge -- and, when the capture's span reaches the
    timeout, the sweep composition.  Every rank ends up holding the final
    records of its own flows; gather_records() collects them on one rank.

    Run the context on torch's current stream (a non-default torch.cuda.Stream
    made current, FlowContext(stream=that_stream.cuda_stream)) so RCCL orders
    the collectives after the export without host waits; a context on a
    stream of its own is synchronised around every collective instead."""

    def __init__(self, ctx, cap: int = 64, cap_annex: int = 16, group=None, wire=None):
        self.ctx, self.group = ctx, group
        self._S = _StepState(cap, cap_annex, wire)
        self._comm = None
        self._rank_first = None

    @property
    def cap(self):
        return self._S.cap

    @property
    def cap_annex(self):
        return self._S.cap_annex

    @property
    def bytes_sent(self):
        """Bytes this rank's last step sent to other ranks in the merge's all-to-all."""
        return self._S.bytes_sent

    @property
    def wire_used(self):
        """The last step moved the compact wire encoding (else equal wide blocks)."""
        return self._S.wire_used

    @property
    def device_agreed(self):
        """The last step was agreed on the device (one host read: the retry word)."""
        return self._S.device_agreed

    @property
    def host_reads(self):
        """Values this rank's collectives read back to the host so far."""
        return self._comm.host_reads if self._comm is not None else 0

    def _rank_first_fn(self):
        if self._rank_first is None:
            comm = self._comm
            mine = np.array([getattr(self.ctx, "index_base", 0), self.ctx.n_packets], dtype=np.int64)
            g = comm.allgather([mine])
            first = [int(x) for x in g[:, 0]]
            total = max(int(a + b) for a, b in g)
            self._rank_first = first + [total]
        return self._rank_first

    def step(self):
        """One sharded pass; this rank's merge stats."""
        if self._comm is None:
            self._comm = _DistComm(self.group, self.ctx)
        (st,) = _shard_step(self._comm, [self.ctx], self._S, self._rank_first_fn)
        return st

    def gather_records(self, dst: int = 0):
        """Every rank's records -> (records, n_ended) on rank dst in the
        reference's order (ended prefix by emission order, then the active
        flows); None elsewhere."""
        import torch.distributed as dist
        recs, _ = self.ctx.records()
        aux = self.ctx.record_order(len(recs))
        parts = [None] * dist.get_world_size(self.group) if dist.get_rank(self.group) == dst else None
        dist.gather_object((recs.tobytes(), aux.tobytes()), parts, dst=dst, group=self.group)
        if parts is None:
            return None
        return order_records([np.frombuffer(p[0], dtype=RECORD_DTYPE) for p in parts],
                             [np.frombuffer(p[1], dtype=np.uint64).reshape(-1, 2) for p in parts])


def order_records(parts, auxes=None):
    """Records of several ranks -> (records, n_ended): ended records by their
    order key (the global index of the packet that ended them, then the sweep
    composition's order words), then active."""
    allr = np.concatenate(parts) if parts else np.zeros(0, dtype=RECORD_DTYPE)
    if auxes is not None and len(auxes):
        aux = np.concatenate([a.reshape(-1, 2) for a in auxes]) if len(allr) else np.zeros((0, 2), np.uint64)
    else:
        aux = np.zeros((len(allr), 2), dtype=np.uint64)
    order = np.lexsort((allr["first"], aux[:, 1], aux[:, 0], allr["order_key"]))
    allr = allr[order]
    return allr, int((allr["order_key"] != NONE64).sum())


class LogicalShards:
    """G shards on one device through the same export / merge / sweep calls,
    with every collective done by device copies (SURVEY.md section 8e "testing
    without 8 GPUs"): contexts[r] holds packets [first_r, first_r + n_r)."""

    def __init__(self, contexts, cap: int = 1024, cap_annex: int = 256, wire=None):
        self.ctxs = contexts
        self._S = _StepState(cap, cap_annex, wire)
        self._comm = _LocalComm(len(contexts))

    @property
    def cap(self):
        return self._S.cap

    @property
    def cap_annex(self):
        return self._S.cap_annex

    @property
    def bytes_sent(self):
        """Bytes shard 0 sent to the other shards in the last step's all-to-all."""
        return self._S.bytes_sent

    @property
    def wire_used(self):
        return self._S.wire_used

    @property
    def device_agreed(self):
        return self._S.device_agreed

    @property
    def host_reads(self):
        return self._comm.host_reads

    def _rank_first(self):
        first = [int(getattr(c, "index_base", 0)) for c in self.ctxs]
        total = max(f + int(c.n_packets) for f, c in zip(first, self.ctxs))
        return first + [total]

    def run(self):
        return _shard_step(self._comm, self.ctxs, self._S, self._rank_first)

    def records(self):
        parts, auxes = [], []
        for c in self.ctxs:
            r, _ = c.records()
            parts.append(r)
            auxes.append(c.record_order(len(r)))
        return order_records(parts, auxes)
