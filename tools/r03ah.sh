#!/bin/bash
# merge owner cap (FLUERE_MAX_OWNERS) on the many-flow configs: hot-kernel / step times
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for c in tcp c4 tcp; do
  for m in 2048 1024 512; do
    export FLUERE_MAX_OWNERS=$m
    out=$(timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config $c 2>&1 | grep '^{')
    echo "$c max_owners=$m $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "step_ms", j["ms_per_step"], "recs", j["records"])')"
  done
done
