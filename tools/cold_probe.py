"""Cold (one-shot) runs of a bench config: fresh context + first fluere_run,
repeated, then a steady rerun on the last context -- the path `fluere offline`
takes.  Run under rocprofv3 --kernel-trace to see the first run's timeline.
  python tools/cold_probe.py [config] [repeats]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import fluere_amd  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "tcp"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
C = bench.CONFIGS[cfg_name]
n = C["per_gpu"]
cfg = fluere_amd.synth_cfg(C["kind"], n, C["flows"], C["seed"])
batches = fluere_amd.synth_device_batches(cfg, 0, n)
torch.cuda.synchronize()
max_flows = max(1 << 16, 2 * C["flows"]) if C["kind"] not in (4, 6) else n // 2
keep = None
if len(sys.argv) > 3 and sys.argv[3] == "keep":  # a steady context stays open (as in bench.py's cold run)
    keep = fluere_amd.FlowContext(timeout_ms=C.get("timeout_ms", 600000), use_mac=C["use_mac"], max_flows=max_flows)
    for b, o, nbytes, nb in batches:
        keep.add_device_batch(b, nbytes, o, nb)
    for _ in range(3):
        keep.run()
    torch.cuda.synchronize()
for r in range(reps):
    print(f"--- rep {r}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    ctx = fluere_amd.FlowContext(timeout_ms=C.get("timeout_ms", 600000), use_mac=C["use_mac"], max_flows=max_flows)
    t1 = time.perf_counter()
    for b, o, nbytes, nb in batches:
        ctx.add_device_batch(b, nbytes, o, nb)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("--- first run", file=sys.stderr, flush=True)
    st = ctx.run()
    t3 = time.perf_counter()
    print("--- rerun", file=sys.stderr, flush=True)
    st2 = ctx.run()
    t4 = time.perf_counter()
    print(f"{cfg_name} rep {r}: open {1e3 * (t1 - t0):.2f} ms attach {1e3 * (t2 - t1):.2f} ms "
          f"first run {1e3 * (t3 - t2):.3f} ms ({ctx.last_hot_kernel()} after; first kernel {st['parse_ms']:.3f}) "
          f"rerun {1e3 * (t4 - t3):.3f} ms kernel {st2['parse_ms']:.3f} records {st['records']} complex "
          f"{st['complex_flows']}", flush=True)
    ctx.close()
