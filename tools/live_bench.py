"""Throughput of live mode on batched capture.

A synthetic capture is cut into batches of --batch packets (classic pcap
images in host memory, as a capture ring delivers them); every --export-every
batches the interval export runs (idle-timeout scan + CSV records).  Times the
fluere_live_batch calls (host pcap -> HBM -> parse / aggregate / compose into
the session's open flows -> exported records back to the host) and the final
flush.  Host-inclusive: the batches start in host memory.

  python tools/live_bench.py [--config c2|tcp] [--packets N] [--batch B] [--export-every K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"c2": (0, 1000, 0xF10E0002), "tcp": (4, 100_000, 0xF10E0007)}
MAX_FLOWS = {"c2": 1 << 16, "tcp": 1 << 21}  # the session's distinct keys over the whole capture


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--export-every", type=int, default=5)
    ap.add_argument("--timeout-ms", type=int, default=600000)
    ap.add_argument("--indexed", type=int, default=1, help="1: batches carry their record offsets")
    args = ap.parse_args()
    import fluere_amd
    from fluere_amd.live import LiveSession, pcap_records

    kind, flows, seed = CONFIGS[args.config]
    data = fluere_amd.synth_pcap(fluere_amd.synth_cfg(kind, args.packets, flows, seed))
    import numpy as np
    hdr = data[:24]
    batches, cur, n = [], [], 0

    def close(cur):
        # the image and its record offsets, as a capture ring hands them over
        lens = np.array([ln for _, ln in cur], dtype=np.uint64)
        offs = 24 + np.concatenate([np.zeros(1, np.uint64), np.cumsum(lens)[:-1]]).astype(np.uint64)
        batches.append((hdr + b"".join(data[o:o + l] for o, l in cur), offs if args.indexed else None))

    for off, ln, _ in pcap_records(data):
        cur.append((off, ln))
        if len(cur) == args.batch:
            close(cur)
            cur = []
    if cur:
        close(cur)
    del data
    res = {"config": args.config, "packets": args.packets, "batch_packets": args.batch, "batches": len(batches),
           "export_every": args.export_every, "indexed": bool(args.indexed), "timeout_ms": args.timeout_ms}
    with LiveSession(args.timeout_ms, False, max_flows=MAX_FLOWS[args.config]) as s:
        s.batch(batches[0][0], False, batches[0][1])  # warm-up (the runtime, the session buffers)
    times, exported = [], 0
    with LiveSession(args.timeout_ms, False, max_flows=MAX_FLOWS[args.config]) as s:
        t_all = time.perf_counter()
        for k, (b, o) in enumerate(batches):
            t0 = time.perf_counter()
            got = s.batch(b, (k + 1) % args.export_every == 0, o)
            times.append(time.perf_counter() - t0)
            if got is not None:
                exported += len(got[0])
        t0 = time.perf_counter()
        recs, _ = s.finish(False)
        t_fin = time.perf_counter() - t0
        total = time.perf_counter() - t_all
    exported += len(recs)
    res.update({"total_s": round(total, 4), "mpps": round(args.packets / total / 1e6, 2),
                "batch_ms_mean": round(1e3 * sum(times) / len(times), 3), "batch_ms_max": round(1e3 * max(times), 3),
                "finish_ms": round(1e3 * t_fin, 3), "records_exported": exported})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
