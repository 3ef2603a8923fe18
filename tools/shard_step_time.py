"""Rank-0 work of the multi-GPU step, timed on one GPU (diagnostics).

The real step (bench.py --gpus N) is: parse+key+aggregate over the shard,
fluere_export_device into a shard block, one all_gather of the blocks (RCCL),
a read of the gathered headers, and fluere_merge_gathered on rank 0.  Here the
all_gather is replaced by device copies of this rank's own block into the N
slots, so the printed time is the step without the collective itself.
  python tools/shard_step_time.py [N] [steps]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import fluere_amd  # noqa: E402
from fluere_amd import _lib  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    L = _lib.lib()
    cfg = fluere_amd.synth_cfg(_lib.SYNTH_UDP64, 10_000_000 * N, 1000, 0xF10E0002)
    b, o, nbytes = fluere_amd.synth_device(cfg, 0, 10_000_000)
    torch.cuda.synchronize()
    ctx = fluere_amd.FlowContext(max_flows=1 << 16, stream=torch.cuda.current_stream().cuda_stream)
    ctx.add_device_batch(b, nbytes, o, 10_000_000)
    cap = 1024
    blk = int(L.fluere_shard_block_bytes(cap))
    send = torch.empty(blk, dtype=torch.uint8, device="cuda")
    recv = torch.empty(N * blk, dtype=torch.uint8, device="cuda")
    merger = fluere_amd.FlowContext(max_flows=1 << 16, stream=torch.cuda.current_stream().cuda_stream)
    t_parts = {"aggregate+export": 0.0, "headers": 0.0, "merge": 0.0}

    def step(timed):
        t0 = time.perf_counter()
        ctx.parse_aggregate()
        _lib.check(L.fluere_export_device(ctx._h, send.data_ptr(), cap), "export")
        recv.view(N, blk).copy_(send.expand(N, blk))  # stands in for the all_gather
        t1 = time.perf_counter()
        n = recv.view(N, blk)[:, :8].contiguous().view(torch.int64).cpu().tolist()
        assert max(int(v[0]) for v in n) <= cap
        t2 = time.perf_counter()
        st = _lib.Stats()
        rc = L.fluere_merge_gathered(merger._h, recv.data_ptr(), N, cap, ctypes.byref(st))
        t3 = time.perf_counter()
        if timed:
            t_parts["aggregate+export"] += t1 - t0
            t_parts["headers"] += t2 - t1
            t_parts["merge"] += t3 - t2
        return rc, st

    for _ in range(3):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        rc, st = step(True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"N={N}: step {dt * 1e3:.3f} ms without the collective (rc {rc}, records {st.records}); "
          + ", ".join(f"{k} {v / steps * 1e3:.3f} ms" for k, v in t_parts.items()))


if __name__ == "__main__":
    main()
