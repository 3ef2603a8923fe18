"""bench.py -- device-resident pcap->flow Mpackets/s on MI355X (BASELINE.json metric).

Step = one pass of the `fluere offline` hot path over one batch of synthetic
pcap records already resident in HBM: parse (parse_keys + parse_fluereflow),
exact flow key, update_flow aggregation and the record finalisation (the
records are materialised in HBM: the reference's "Converted in" window also
ends before the CSV export, offline_fluereflows.rs:178).  For N > 1 each rank
aggregates its shard and the step adds the flow-table merge: every rank
exports its flows into one block per owner rank, one RCCL all_to_all over
xGMI, and each owner merges / finalizes its own flows (fluere_amd/dist.py).
Weak scaling: every rank owns a fixed per-GPU shard of one global capture
(packet-range sharding with global packet indices); c4 (BASELINE configs[3],
a fixed 100M-packet capture) scales strong: N ranks share its packets.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c4_shard|c5|c5u|tcp|tcp_t1|tcp_t1_backtime|slow]
  torchrun --nproc-per-node N bench.py --gpus N ...   (N > 1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# per-GPU workload of each BASELINE config
CONFIGS = {
    "c2": dict(kind=0, per_gpu=10_000_000, flows=1000, seed=0xF10E0002, use_mac=False,
               workload="10M x 64B UDP, 1k 5-tuples per GPU (BASELINE configs[1])"),
    "c3": dict(kind=1, per_gpu=10_000_000, flows=100_000, seed=0xF10E0003, use_mac=False,
               workload="10M IMIX 64/576/1500 TCP+UDP, 100k flows per GPU (BASELINE configs[2])"),
    # BASELINE configs[3]: 100M IMIX packets, 1M flows, sharded across 2/4/8
    # GPUs -- a fixed capture (strong scaling: N ranks take 100M / N packets
    # each); the flow count is global, so every shard sees nearly all 1M flows
    "c4": dict(kind=1, total=100_000_000, flows=1_000_000, seed=0xF10E0004, use_mac=False,
               workload="100M IMIX TCP+UDP packets, 1M flows, sharded over the GPUs (BASELINE configs[3])"),
    # one 8-GPU shard of it on one GPU (the per-GPU work of c4 at N = 8; weak)
    "c4_shard": dict(kind=1, per_gpu=12_500_000, flows=1_000_000, seed=0xF10E0004, use_mac=False,
                     workload="IMIX TCP+UDP, 12.5M packets per GPU, 1M flows in the whole capture "
                              "(BASELINE configs[3]'s per-GPU shard at N = 8)"),
    "c5": dict(kind=2, per_gpu=10_000_000, flows=50_000, seed=0xF10E0005, use_mac=True,
               workload="10M x 64B VLAN-tagged, 50k MAC pairs, --useMAC (BASELINE configs[4]; header-only CSV)",
               note="drop-only path: the reference's vlan_keys misparse (keys.rs:417-435) skips every frame, "
                    "so no packet is aggregated; see c5u for MAC-keyed aggregation"),
    "c5u": dict(kind=3, per_gpu=10_000_000, flows=50_000, seed=0xF10E0005, use_mac=True,
                workload="10M x 64B untagged, 50k MAC pairs, --useMAC (BASELINE configs[4], untagged)"),
    # realistic TCP (FLUERE_SYNTH_TCP): 4-way closes, RSTs, reopened keys,
    # mid-stream starts, elephants -- the exact state machine (exact.hip) runs
    # for every flow the certificate rejects; with -t 1000 (1 s, the capture
    # spans 10 s) the hard-timeout sweep runs for every flow (Mode B)
    "tcp": dict(kind=4, per_gpu=10_000_000, flows=100_000, seed=0xF10E0007, use_mac=False,
                workload="10M IMIX, realistic TCP (+UDP), 100k concurrent lanes, -t 600000"),
    # the general parser's classes: every packet takes the slow
    # list (parsed in k_merge_partials' tail, pre-aggregated per dense id in LDS)
    "slow": dict(kind=5, per_gpu=10_000_000, flows=10_000, seed=0xF10E0008, use_mac=False,
                 workload="10M general-parser packets at 128/576/1500 B (IPv6 1/2, VXLAN 1/4, IPv4 options 1/4), "
                          "10k flows"),
    "tcp_t1": dict(kind=4, per_gpu=10_000_000, flows=100_000, seed=0xF10E0007, use_mac=False, timeout_ms=1000,
                   workload="10M IMIX, realistic TCP (+UDP), 100k concurrent lanes, -t 1000 (expiry sweep)"),
    # the same with 1 % of the timestamps up to 5 ms early (merged / multi-queue
    # captures): the sweep points from the max segment tree
    "tcp_t1_backtime": dict(kind=6, per_gpu=10_000_000, flows=100_000, seed=0xF10E0047, use_mac=False,
                            timeout_ms=1000,
                            workload="10M IMIX, realistic TCP (+UDP), 100k lanes, 1% timestamps up to 5 ms early, "
                                     "-t 1000 (expiry sweep, out-of-order times)"),
}
BYTES_PER_PKT = 80  # algorithmic: 16 B pcap record header + min(caplen, 64) B header window
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0  # measured device copy rate (MI355X_MICROARCH.md)


def packets_total(C, world):
    """Packets of the whole job: a fixed capture shared by the ranks (strong,
    c4), else the per-GPU shard times the ranks (weak)."""
    return C["total"] if "total" in C else C["per_gpu"] * world


def measure(name, args, world, rank, local, stream, torch, dist, fluere_amd, fdist):
    """Warmup + timed steps of one config on this rank; every rank returns its
    numbers, the max over ranks already taken for the times."""
    C = CONFIGS[name]
    n_total = packets_total(C, world)
    cfg = fluere_amd.synth_cfg(C["kind"], n_total, C["flows"], C["seed"])
    first, n = fdist.shard_range(n_total, rank, world)

    # synthetic capture generated directly in HBM (untimed), as batches below
    # 4 GiB each (u32 record offsets; a C4 IMIX shard is ~4.4 GB)
    batches = fluere_amd.synth_device_batches(cfg, first, n)
    torch.cuda.synchronize()
    max_flows = max(1 << 16, 2 * C["flows"]) if C["kind"] not in (4, 6) else n // 2
    ctx = fluere_amd.FlowContext(timeout_ms=C.get("timeout_ms", 600000), use_mac=C["use_mac"], max_flows=max_flows,
                                 device=local, stream=stream)
    exchange = fdist.ShardExchange(ctx) if world > 1 else None
    fdist.set_index_base(ctx, first)
    for b, o, nbytes, nb in batches:
        ctx.add_device_batch(b, nbytes, o, nb)

    kernel_ms, pass_ms = [], []

    def step():
        if world == 1:
            # parse + key + aggregate + finalize + the ended records ordered
            # on the device; the records stay in HBM
            st = ctx.run()
        else:
            # per-shard aggregation, then the flow-table merge: per-owner
            # blocks, one RCCL all_to_all, each owner merges its own flows
            st = exchange.step()
        # HIP events carried by the hot-kernel dispatches on the context stream,
        # summed over the step's launches (fluere_stats.parse_ms)
        kernel_ms.append(st["parse_ms"] if world == 1 else ctx.last_kernel_ms())
        pass_ms.append(st["total_ms"] if world == 1 else ctx.last_pass_ms())
        return st

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    kernel_ms.clear()
    pass_ms.clear()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([sum(kernel_ms) / len(kernel_ms)], dtype=torch.float64, device="cuda")
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_avg = float(km.item())
    else:
        kernel_avg = sum(kernel_ms) / len(kernel_ms)

    # the one-shot seam (`fluere offline` converts a capture once): a fresh
    # context on the same resident batches, its first run timed on the host
    # (the census, every allocation and choice the first run makes included)
    cold = cold_run(fluere_amd, batches, C, max_flows, local) if world == 1 and not args.no_cold else {}

    # records of the whole job: every rank holds its own flows' records
    recs, ne = ctx.records()
    n_recs, n_ended = len(recs), ne
    if world > 1:
        t = torch.tensor([n_recs, n_ended], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        n_recs, n_ended = (int(x) for x in t.tolist())
    ms_per_step = 1e3 * elapsed / args.steps
    achieved = BYTES_PER_PKT * n / (kernel_avg * 1e-3) / 1e9  # per-GPU launch (GB/s)
    traffic = None
    prof = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if os.path.exists(prof):
        traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
    out = dict(
        C=C, cfg=cfg, n=n, n_total=n_total, ms_per_step=ms_per_step, mpps=n_total / (elapsed / args.steps) / 1e6,
        kernel_avg=kernel_avg, achieved=achieved, traffic=traffic, kernel=ctx.last_hot_kernel(),
        launches=len(batches), pass_ms=sum(pass_ms) / len(pass_ms), n_recs=n_recs, n_ended=n_ended, st=st,
        exchange_bytes=int(exchange.bytes_sent) if world > 1 else None, cold=cold)
    ctx.close()
    del batches
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def roofline(m):
    return {"bound": "hbm", "achieved": round(m["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(m["achieved"] / HBM_PEAK_GBS, 4), "traffic": m["traffic"],
            # also against the measured copy rate (MI355X_MICROARCH.md)
            "frac_vs_copy_6290": round(m["achieved"] / HBM_COPY_GBS, 4),
            # kernel_ms: the step's hot-kernel launches, their device times summed
            # (HIP events carried by each dispatch); per launch: divided by their count
            "kernel": m["kernel"], "kernel_ms": round(m["kernel_avg"], 4),
            "launches_per_step": m["launches"],
            "kernel_ms_per_launch": round(m["kernel_avg"] / max(1, m["launches"]), 4),
            "algorithmic_bytes_per_launch": BYTES_PER_PKT * m["n"] // max(1, m["launches"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-imix", action="store_true", help="default line without its IMIX (c3) object")
    ap.add_argument("--no-cold", action="store_true", help="skip the one-shot (fresh context) run")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import fluere_amd
    from fluere_amd import dist as fdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        # one process per GPU; "nccl" is RCCL on ROCm.  FLUERE_DIST_BACKEND=gloo
        # rehearses the sharded path with several ranks on one GPU (tests only).
        backend = os.environ.get("FLUERE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    # N > 1: the context runs on torch's current stream (a stream of its own,
    # not the null stream, made current), so RCCL orders the shard exchange's
    # collectives after the export without a host wait
    stream = None
    if world > 1:
        ts = torch.cuda.Stream()
        torch.cuda.set_stream(ts)
        stream = ts.cuda_stream
    mods = (torch, dist, fluere_amd, fdist)
    m = measure(args.config, args, world, rank, local, stream, *mods)
    # the metric is "64B & IMIX": the default (64-B, c2) line carries the IMIX
    # config (c3) measured the same way in the same run
    imix = None
    if args.config == "c2" and not args.no_imix:
        imix = measure("c3", args, world, rank, local, stream, *mods)
    if rank == 0:
        C, st = m["C"], m["st"]
        line = {
            "metric": "Mpackets/s device-resident pcap->flow parse+key, 64B & IMIX, 1/2/4/8 GPU",
            "value": round(m["mpps"], 1),
            "unit": "Mpackets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(m["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "strong" if "total" in C else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-based generator, device-resident)",
            "config": {"workload": C["workload"], "packets_total": m["n_total"], "flows": C["flows"],
                       "parallelism": (f"dp{world}: packet-range shards, owner-partitioned flow-table merge "
                                       "(one RCCL all_to_all of per-owner blocks)"
                                       if world > 1 else "single GPU"),
                       "use_mac": C["use_mac"], "timeout_ms": C.get("timeout_ms", 600000),
                       **({"note": C["note"]} if "note" in C else {})},
            "roofline": roofline(m),
            "parse_key_mpps_per_gpu": round(m["n"] / (m["kernel_avg"] * 1e-3) / 1e6, 1),
            "aggregate_pass_ms": round(m["pass_ms"], 4),
            "records": int(m["n_recs"]),
            "records_ended": int(m["n_ended"]),
            # the step ends with the ended records in the reference's order, on the device
            "ordering": "ended records ordered on the device inside the step" if world == 1 else
                        "per owner rank; merged across ranks on fetch",
            "complex_flows": int(st.get("complex_flows", 0)) if world == 1 else None,
            # N > 1: bytes each rank sends to the others in the merge's all-to-all
            "exchange_bytes_per_rank": m["exchange_bytes"],
            "sequential_mode": int(st.get("sequential_mode", 0)) if world == 1 else None,
            "exact_passes": int(st.get("passes", 0)) if world == 1 else None,
            **m["cold"],
        }
        if imix is not None:
            line["imix"] = {"workload": imix["C"]["workload"], "packets_total": imix["n_total"],
                            "value": round(imix["mpps"], 1), "unit": "Mpackets/s",
                            "ms_per_step": round(imix["ms_per_step"], 4), "kernel": imix["kernel"],
                            "kernel_ms": round(imix["kernel_avg"], 4),
                            "frac": round(imix["achieved"] / HBM_PEAK_GBS, 4), "traffic": imix["traffic"],
                            "records": int(imix["n_recs"]), "records_ended": int(imix["n_ended"]),
                            "roofline": roofline(imix), **imix["cold"]}
            if world == 1 and not args.no_cpu_baseline:
                line["imix"]["cpu_baseline"] = cpu_baseline(imix["cfg"], imix["C"])
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(m["cfg"], C)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def cold_run(fluere_amd, batches, C, max_flows, device):
    """Fresh FlowContext + attach + first fluere_run, host wall clock: the path
    `fluere offline` takes (one run per context).  cold_run_ms is the first run
    alone; cold_open_attach_ms the open and the attach, which runs the census
    of the capture and reserves the buffers it implies (fluere_add_*)."""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx = fluere_amd.FlowContext(timeout_ms=C.get("timeout_ms", 600000), use_mac=C["use_mac"], max_flows=max_flows,
                                 device=device)
    for b, o, nbytes, nb in batches:
        ctx.add_device_batch(b, nbytes, o, nb)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    st = ctx.run()
    t2 = time.perf_counter()
    out = {"cold_run_ms": round(1e3 * (t2 - t1), 4), "cold_open_attach_ms": round(1e3 * (t1 - t0), 3),
           "cold_total_ms": round(1e3 * (t2 - t0), 3),
           "cold_hot_kernel": ctx.last_hot_kernel(), "cold_kernel_ms": round(st["parse_ms"], 4)}
    ctx.close()
    return out


def cpu_baseline(cfg, C):
    """The oracle (C restatement of the reference CPU path, single thread, pinned
    to one core) over the same workload, timed over the reference's "Converted in"
    window (pcap open -> end of packet loop, offline_fluereflows.rs:49,178)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fluere_amd
    import pyoracle
    n = min(cfg.n_packets, 4_000_000)
    sample = fluere_amd.synth_cfg(cfg.kind, n, cfg.n_flows, cfg.seed)
    data = fluere_amd.synth_pcap(sample)
    old = os.sched_getaffinity(0)
    try:
        os.sched_setaffinity(0, {sorted(old)[0]})
        best = min(pyoracle.offline(data, C.get("timeout_ms", 600000), use_mac=C["use_mac"])["loop_seconds"]
                   for _ in range(2))
    finally:
        os.sched_setaffinity(0, old)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": round(n / best / 1e6, 3), "unit": "Mpackets/s", "cores": 1, "kind": "port",
            "sample": f"first {n} packets of the same synthetic capture, in memory, best of 2",
            "what": "C restatement of the reference CPU path (oracle/), 1 core; the Rust reference cannot be built here",
            "cpu": model, "host_cpus": os.cpu_count()}


if __name__ == "__main__":
    main()
