#!/bin/bash
# C2 merge diagnostics: FLUERE_DEBUG phases and the step timeline
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03ak; mkdir -p $O
cd $R
FLUERE_DEBUG=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --config c2 > $O/dbg_c2.log 2>&1
grep -E "merge|WG starts" $O/dbg_c2.log | tail -4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_c2" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --config c2 > "$O/tr_c2.log" 2>&1
f=$(find "$O/tr_c2" -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline_last.py "$f" k_parse > $O/timeline_c2.txt
find "$O/tr_c2" -type f -size +1M -delete
cat $O/timeline_c2.txt
