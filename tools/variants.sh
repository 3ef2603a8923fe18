#!/bin/bash
# Time k_parse_agg variants on C2: FLUERE_PIPE x FLUERE_ABLATE (diagnostics).
#   tools/variants.sh "1 3" "0 1" [config]
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=${3:-c2}
for p in $1; do
  for a in $2; do
    out=$(FLUERE_PIPE=$p FLUERE_ABLATE=$a timeout -k 10 120 python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --config "$CFG" 2>&1 | grep '^{') || { echo "pipe=$p abl=$a FAILED"; exit 1; }
    echo "pipe=$p abl=$a $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "GB/s", j["roofline"]["achieved"], "step_ms", j["ms_per_step"])')"
  done
done
