#!/bin/bash
# Round 3: rocprofv3 kernel stats of the bench workloads (one run each).
#   tools/r03prof.sh <tag> <config> [<config> ...]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
for CFG in "$@"; do
  O=$R/gpurun_out/prof_${TAG}_$CFG
  mkdir -p "$O"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --config "$CFG" > "$O/trace.log" 2>&1
  f=$(find "$O/trace" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/kernel_stats.csv"
  find "$O/trace" -type f -size +1M -delete
  python3 - "$O/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    n = r["Name"]
    n = n[n.find("k_"):][:60] if "k_" in n else n[:60]
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {n}')
PY
  tail -1 "$O/trace.log" | cut -c1-200
done
