#!/bin/bash
# rocprofv3 kernel statistics of the default bench command (C2 line with its
# IMIX object and cold runs; no CPU baseline): gpurun_out/prof_default/
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/prof_default
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench.log" 2>&1
f=$(find "$O/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$O/kernel_stats.csv"
find "$O/trace" -type f -size +1M -delete
tail -1 "$O/bench.log" | cut -c1-200
