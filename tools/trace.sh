#!/bin/bash
# Kernel-trace one bench config and print the step timeline (diagnostics).
#   tools/trace.sh <tag> [config]  -> gpurun_out/trace_<tag>/
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
TAG=${1:-x}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/trace_$TAG
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --config "$CFG" > "$O/trace.log" 2>&1
f=$(find "$O" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline.py" "$f" 16 > "$O/timeline.txt"
cat "$O/timeline.txt"
