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
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import RECORD_DTYPE, Stats, check


def shard_range(n_packets: int, rank: int, world: int):
    per = (n_packets + world - 1) // world
    first = min(n_packets, rank * per)
    return first, min(n_packets, first + per) - first


def set_index_base(ctx, base: int):
    check(_lib.lib().fluere_set_index_base(ctx._h, base), "fluere_set_index_base")


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


class ShardExchange:
    """The multi-GPU step: parse + key + aggregate over this rank's shard,
    export into per-owner blocks (summaries of every flow, annexes of the flows
    whose record depends on packet order in this shard, whose records that
    open and close inside the shard stay here), agree on the block capacities,
    one all-to-all, owner merge.  Every rank ends up holding the final records
    of its own flows; gather_records() collects them on one rank.

    The context must run on torch's current stream (FlowContext(stream=
    torch.cuda.current_stream().cuda_stream)) so the collective is ordered
    after the export."""

    def __init__(self, ctx, cap: int = 64, cap_annex: int = 16, group=None):
        self.ctx, self.group = ctx, group
        self.cap, self.cap_annex = max(1, int(cap)), max(1, int(cap_annex))
        self._send = self._recv = None
        self._info = None

    def _buffers(self, world, device):
        import torch
        blk = int(_lib.lib().fluere_shard_block_bytes(self.cap, self.cap_annex))
        if self._send is None or self._send.numel() != world * blk or self._send.device != device:
            self._send = torch.empty(world * blk, dtype=torch.uint8, device=device)
            self._recv = torch.empty(world * blk, dtype=torch.uint8, device=device)
        return blk

    def step(self, allow_unsupported: bool = False):
        """One sharded pass; this rank's merge stats.  Raises FluereError when
        the merge cannot give the exact result (FLUERE_E_UNSUPPORTED: the
        capture needs the hard-timeout sweep) unless allow_unsupported.

        Common case: two host round trips per step -- the export (summaries,
        no annexes) and a MAX all-reduce of its counts are enqueued behind the
        pass and read once, then the all-to-all and the owner merge.  If any
        rank has order-dependent flows, every rank exports again with annexes
        (fluere_export_device); if a block was too small, every rank exports
        again with larger blocks."""
        import torch
        import torch.distributed as dist
        L = _lib.lib()
        ctx = self.ctx
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        dev = torch.device("cuda", torch.cuda.current_device())
        gloo = dist.get_backend(self.group) == "gloo"
        if self._info is None:
            self._info = torch.zeros(4, dtype=torch.int64, device=dev)
        ctx.parse_aggregate()
        annexes = False
        while True:
            self._buffers(world, dev)
            if not annexes:
                check(L.fluere_export_async(ctx._h, self._send.data_ptr(), world, rank, self.cap, self.cap_annex,
                                            self._info.data_ptr()), "fluere_export_async")
                if gloo:  # host copy (the context may run on a stream of its own here)
                    torch.cuda.synchronize()
                    t = self._info.cpu()
                else:     # RCCL on torch's stream, which is the context's (see the class note)
                    t = self._info
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
                n0, n1, n_cplx, _ = (int(x) for x in t.tolist())
                if n_cplx:
                    annexes = True  # some rank has order-dependent flows: export with annexes
                    continue
            else:
                need, need_a = ctypes.c_uint64(), ctypes.c_uint64()
                check(L.fluere_export_device(ctx._h, self._send.data_ptr(), world, rank, self.cap, self.cap_annex,
                                             ctypes.byref(need), ctypes.byref(need_a)), "fluere_export_device")
                n0, n1 = agree_need(need.value, need_a.value, self.group, dev)
            if n0 <= self.cap and n1 <= self.cap_annex:
                break
            # a shard had more flows for some owner: grow the blocks, export again
            self.cap = _pow2_at_least(n0, self.cap)
            self.cap_annex = _pow2_at_least(n1, self.cap_annex)
        exchange_blocks(self._send, self._recv, self.group)
        st = Stats()
        rc = L.fluere_merge_gathered(ctx._h, self._recv.data_ptr(), world, self.cap, self.cap_annex,
                                     ctypes.byref(st))
        if rc != _lib.E_UNSUPPORTED or not allow_unsupported:
            check(rc, "fluere_merge_gathered")
        d = st.as_dict()
        d["rc"] = rc
        return d

    def gather_records(self, dst: int = 0):
        """Every rank's records -> (records, n_ended) on rank dst in the
        reference's order (ended prefix by emission order, then the active
        flows); None elsewhere."""
        import torch.distributed as dist
        recs, _ = self.ctx.records()
        parts = [None] * dist.get_world_size(self.group) if dist.get_rank(self.group) == dst else None
        dist.gather_object(recs.tobytes(), parts, dst=dst, group=self.group)
        if parts is None:
            return None
        return order_records([np.frombuffer(p, dtype=RECORD_DTYPE) for p in parts])


NONE64 = (1 << 64) - 1


def order_records(parts):
    """Records of several ranks -> (records, n_ended): ended records by their
    order key (the global index of the packet that ended them), then active."""
    allr = np.concatenate(parts) if parts else np.zeros(0, dtype=RECORD_DTYPE)
    order = np.lexsort((allr["first"], allr["order_key"]))
    allr = allr[order]
    return allr, int((allr["order_key"] != NONE64).sum())


class LogicalShards:
    """G shards on one device through the same export / merge code, with the
    all-to-all done by device copies (SURVEY.md section 8e "testing without 8
    GPUs"): contexts[r] holds packets [first_r, first_r + n_r)."""

    def __init__(self, contexts, cap: int = 1024, cap_annex: int = 256):
        self.ctxs = contexts
        self.cap, self.cap_annex = cap, cap_annex

    def run(self, allow_unsupported: bool = False):
        import torch
        L = _lib.lib()
        G = len(self.ctxs)
        for c in self.ctxs:
            c.parse_aggregate()
        while True:
            blk = int(L.fluere_shard_block_bytes(self.cap, self.cap_annex))
            sends, n0, n1 = [], 0, 0
            for r, c in enumerate(self.ctxs):
                send = torch.empty(G * blk, dtype=torch.uint8, device="cuda")
                need, need_a = ctypes.c_uint64(), ctypes.c_uint64()
                check(L.fluere_export_device(c._h, send.data_ptr(), G, r, self.cap, self.cap_annex,
                                             ctypes.byref(need), ctypes.byref(need_a)), "fluere_export_device")
                sends.append(send)
                n0, n1 = max(n0, need.value), max(n1, need_a.value)
            if n0 <= self.cap and n1 <= self.cap_annex:
                break
            self.cap = _pow2_at_least(n0, self.cap)
            self.cap_annex = _pow2_at_least(n1, self.cap_annex)
        torch.cuda.synchronize()
        stats = []
        for o, c in enumerate(self.ctxs):
            recv = torch.cat([s[o * blk:(o + 1) * blk] for s in sends])
            # the contexts run on streams of their own: the copy must have landed
            torch.cuda.current_stream().synchronize()
            st = Stats()
            rc = L.fluere_merge_gathered(c._h, recv.data_ptr(), G, self.cap, self.cap_annex, ctypes.byref(st))
            if rc != _lib.E_UNSUPPORTED or not allow_unsupported:
                check(rc, "fluere_merge_gathered")
            stats.append(st.as_dict())
        return stats

    def records(self):
        return order_records([c.records()[0] for c in self.ctxs])
