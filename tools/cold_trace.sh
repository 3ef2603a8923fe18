#!/bin/bash
# Kernel trace of cold runs (fresh contexts, a steady context kept open as in
# bench.py): the last 160 kernels = the last context's first run and rerun.
#   tools/cold_trace.sh <config>
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${1:-c3}
O=$R/gpurun_out/coldtrace_$C
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/tr" -o run -- \
  python3 "$R/tools/cold_probe.py" $C 2 keep > "$O/run.log" 2>&1
f=$(find "$O/tr" -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py "$f" 160 > $O/timeline.txt
find "$O/tr" -type f -size +1M -delete
grep "rep" "$O/run.log"
