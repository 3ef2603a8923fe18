#!/bin/bash
# Kernel timelines of one bench config under two environments (A/B):
#   tools/ab_trace.sh <tag> <config> <VAR=a> <VAR=b>  -> gpurun_out/<tag>/timeline_<config>_<a|b>.txt
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; CFG=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
for kv in "$@"; do
  env "$kv" bash "$R/tools/trace.sh" "${TAG}_${kv//=/_}" "$CFG"
  cp "$R/gpurun_out/trace_${TAG}_${kv//=/_}_$CFG/timeline.txt" "$O/timeline_${CFG}_${kv//=/_}.txt"
  f=$(find "$R/gpurun_out/trace_${TAG}_${kv//=/_}_$CFG" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/kernel_stats_${CFG}_${kv//=/_}.csv"
done
