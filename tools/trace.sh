#!/bin/bash
# Kernel-trace one bench config and print the last step's timeline (diagnostics).
#   tools/trace.sh <tag> [config]  -> gpurun_out/trace_<tag>_<config>/
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
TAG=${1:-x}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/trace_${TAG}_$CFG
mkdir -p "$O"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O" -o run -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline --no-imix --no-cold --config "$CFG" > "$O/trace.log" 2>&1
f=$(find "$O" -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/timeline_last.py" "$f" k_parse > "$O/timeline.txt"
find "$O" -type f -name "*kernel_trace.csv" -size +1M -delete
tail -1 "$O/timeline.txt"
