"""Diagnostics: time k_parse_agg ablation variants (FLUERE_ABLATE) on the C2 workload."""
import os, sys, subprocess, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
res = {}
for abl in [int(x) for x in (sys.argv[1:] or ["0", "1", "2", "3"])]:
    env = dict(os.environ, FLUERE_ABLATE=str(abl))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10", "--warmup", "3",
                          "--no-cpu-baseline"], env=env, capture_output=True, text=True)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(abl, out.stderr[-2000:]); continue
    j = json.loads(line[-1])
    res[abl] = j["roofline"]["kernel_ms"]
    print(f"ablate={abl} kernel_ms={j['roofline']['kernel_ms']} GB/s={j['roofline']['achieved']}", flush=True)
