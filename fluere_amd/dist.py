"""Packet-range sharding over GPUs: one process per GPU (torch.distributed,
backend "nccl" = RCCL on ROCm), flow-table merge as one all_gather of per-flow
summaries over xGMI followed by a device merge on rank 0.

Reference: the offline loop is one sequential pass (offline_fluereflows.rs:68-176);
shard r processes packets [r*N/G, (r+1)*N/G) with global packet indices, so the
order-dependent record fields (first / last packet, FIN/RST position) merge as
min / max of global indices.
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import SHARD_HEADER_BYTES, SUMMARY_BYTES, Stats, check


def shard_range(n_packets: int, rank: int, world: int):
    per = (n_packets + world - 1) // world
    first = min(n_packets, rank * per)
    return first, min(n_packets, first + per) - first


def set_index_base(ctx, base: int):
    check(_lib.lib().fluere_set_index_base(ctx._h, base), "fluere_set_index_base")


ONE_PASS_BYTES = 256 << 20  # export buffers up to this size hold every possible flow


def export_summaries(ctx, out=None):
    """parse+key+aggregate this shard and export its flows -> (uint8 cuda tensor [n*192], tmin, tmax).

    With a buffer for the context's whole flow capacity the export is one pass
    with a single host round trip (fluere_capacity).  The buffer is cached on
    the context unless `out` is given; the returned tensor is a view of it."""
    import torch
    L = _lib.lib()
    ctx.parse_aggregate()
    n, lo, hi = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    cap = int(L.fluere_capacity(ctx._h))
    if out is None:
        out = getattr(ctx, "_export_buf", None)
    if cap * SUMMARY_BYTES <= ONE_PASS_BYTES:
        if out is None or out.numel() < cap * SUMMARY_BYTES:
            out = torch.empty(max(cap, 1) * SUMMARY_BYTES, dtype=torch.uint8, device="cuda")
        ctx._export_buf = out
        check(L.fluere_export_summaries(ctx._h, out.data_ptr(), cap, ctypes.byref(n), ctypes.byref(lo),
                                        ctypes.byref(hi)), "fluere_export_summaries")
        return out[: n.value * SUMMARY_BYTES], lo.value, hi.value
    check(L.fluere_export_summaries(ctx._h, None, 0, ctypes.byref(n), ctypes.byref(lo), ctypes.byref(hi)),
          "fluere_export_summaries")
    if out is None or out.numel() < n.value * SUMMARY_BYTES:
        out = torch.empty(max(n.value, 1) * SUMMARY_BYTES, dtype=torch.uint8, device="cuda")
    ctx._export_buf = out
    check(L.fluere_export_summaries(ctx._h, out.data_ptr(), n.value, ctypes.byref(n), None, None),
          "fluere_export_summaries")
    return out[: n.value * SUMMARY_BYTES], lo.value, hi.value


def merge_summaries(ctx, summaries, tmin: int, tmax: int) -> dict:
    st = Stats()
    n = summaries.numel() // SUMMARY_BYTES
    check(_lib.lib().fluere_merge_summaries(ctx._h, summaries.data_ptr() if n else None, n, tmin, tmax,
                                            ctypes.byref(st)), "fluere_merge_summaries")
    return st.as_dict()


NONE64 = (1 << 64) - 1  # tmin of a shard without valid packets


def gather_summaries(summaries, tmin: int, tmax: int, group=None, dst: int = 0):
    """All-gather every shard's flow summaries (RCCL over xGMI on GPUs, gloo on
    CPU) -> (concatenated summaries in rank order, global tmin, global tmax) on
    rank dst, None elsewhere.  Shards may be empty (tmin NONE64)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    out_dev = summaries.device
    # RCCL moves device tensors over xGMI; gloo (CPU tests, rehearsals) moves host copies
    if dist.get_backend(group) == "gloo" and summaries.is_cuda:
        summaries = summaries.cpu()
    dev = summaries.device
    # timestamps are microseconds (< 2^63); an empty shard travels as -1
    meta = torch.tensor([summaries.numel() // SUMMARY_BYTES, tmin if tmin < (1 << 63) else -1, tmax],
                        dtype=torch.int64, device=dev)
    metas = torch.empty(world * 3, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(metas, meta, group=group)
    m = metas.view(world, 3).cpu().tolist()  # one device->host copy
    counts = [int(r[0]) for r in m]
    lows = [int(r[1]) for r in m if int(r[1]) >= 0]
    gmin = min(lows) if lows else NONE64
    gmax = max(int(r[2]) for r in m)
    cap = max(max(counts), 1) * SUMMARY_BYTES
    send = torch.zeros(cap, dtype=torch.uint8, device=dev)
    send[: summaries.numel()] = summaries
    recv = torch.empty(world * cap, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(recv, send, group=group)
    if rank != dst:
        return None
    parts = [recv[r * cap: r * cap + counts[r] * SUMMARY_BYTES] for r in range(world)]
    return torch.cat(parts).to(out_dev), gmin, gmax


def gather_and_merge(ctx, summaries, tmin: int, tmax: int, group=None, dst: int = 0):
    """All-gather every shard's summaries and merge them on rank dst (device
    merge, fluere_merge_summaries).  Returns the merge stats on dst, None
    elsewhere."""
    import torch
    got = gather_summaries(summaries, tmin, tmax, group, dst)
    if got is None:
        return None
    allsum, gmin, gmax = got
    torch.cuda.current_stream().synchronize()  # the collective ran on torch's stream, the merge runs on ctx's
    return merge_summaries(ctx, allsum, gmin, gmax)


class ShardExchange:
    """The multi-GPU step without host round trips in the middle: every rank
    runs parse+key+aggregate over its shard and exports its flows into one
    shard block (fluere_shard_header + `cap` summaries) on the device; one
    all_gather moves the blocks (RCCL over xGMI); rank `dst` merges them on the
    device (fluere_merge_gathered).  The only host reads are the gathered
    headers (every rank checks that no shard had more than `cap` flows, and
    grows `cap` and exchanges again if one had) and the merge's counters.

    The context must run on torch's current stream (FlowContext(stream=
    torch.cuda.current_stream().cuda_stream)) so the collective is ordered
    after the export; otherwise the context stream is synchronised first."""

    def __init__(self, ctx, cap: int = 1024, group=None, dst: int = 0):
        self.ctx, self.cap, self.group, self.dst = ctx, max(1, int(cap)), group, dst
        self._send = self._recv = None

    def _buffers(self, world, device):
        import torch
        blk = int(_lib.lib().fluere_shard_block_bytes(self.cap))
        if self._send is None or self._send.numel() != blk or self._send.device != device:
            self._send = torch.empty(blk, dtype=torch.uint8, device=device)
            self._recv = torch.empty(world * blk, dtype=torch.uint8, device=device)
        return blk

    def step(self, allow_unsupported: bool = False):
        """One sharded pass; the merge stats on rank dst, None elsewhere.
        Raises FluereError when the merge cannot give the exact result
        (FLUERE_E_UNSUPPORTED) unless allow_unsupported."""
        import torch
        import torch.distributed as dist
        L = _lib.lib()
        ctx = self.ctx
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        gloo = dist.get_backend(self.group) == "gloo"
        ctx.parse_aggregate()
        while True:
            blk = self._buffers(world, torch.device("cuda", torch.cuda.current_device()))
            check(L.fluere_export_device(ctx._h, self._send.data_ptr(), self.cap), "fluere_export_device")
            if ctx.stream is None or ctx.stream != torch.cuda.current_stream().cuda_stream:
                torch.cuda.synchronize()  # the export ran on the context's own stream
            if gloo:  # CPU rehearsal: host copies
                recv_h = torch.empty(world * blk, dtype=torch.uint8)
                dist.all_gather_into_tensor(recv_h, self._send.cpu(), group=self.group)
                self._recv.copy_(recv_h)
            else:
                dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
            # the headers' flow counts (one small device->host copy)
            n = self._recv.view(world, blk)[:, :8].contiguous().view(torch.int64).cpu().tolist()
            need = max(int(v[0]) for v in n)
            if need <= self.cap:
                break
            while self.cap < need:  # a shard had more flows: grow the blocks, exchange again
                self.cap *= 2
        if rank != self.dst:
            return None
        st = Stats()
        rc = L.fluere_merge_gathered(ctx._h, self._recv.data_ptr(), world, self.cap, ctypes.byref(st))
        if rc != _lib.E_UNSUPPORTED or not allow_unsupported:
            check(rc, "fluere_merge_gathered")
        d = st.as_dict()
        d["rc"] = rc
        return d
