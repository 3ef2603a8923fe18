#!/bin/bash
# Timeline of the last realistic-TCP step (Mode A) and of -t 1000 (Mode B)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03ad; mkdir -p $O
for CFG in tcp tcp_t1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_$CFG" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --config "$CFG" > "$O/$CFG.log" 2>&1
  f=$(find "$O/tr_$CFG" -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline_last.py "$f" k_parse > $O/timeline_$CFG.txt
  find "$O/tr_$CFG" -type f -size +1M -delete
  cat $O/timeline_$CFG.txt
done
