#!/bin/bash
# Cold-run baseline: host breakdown per config, and a kernel trace of cold tcp runs.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_cold
mkdir -p "$O"
cd "$R"
for c in c2 c3 tcp slow tcp_t1 c5u; do
  FLUERE_HOSTPROF=1 timeout -k 10 120 python -u tools/cold_probe.py $c 2 > "$O/cold_$c.log" 2>&1
  grep rep "$O/cold_$c.log"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_tcp" -o run -- \
  python3 "$R/tools/cold_probe.py" tcp 2 > "$O/tr_tcp.log" 2>&1
f=$(find "$O/tr_tcp" -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py "$f" 400 > $O/timeline_tcp.txt
find "$O/tr_tcp" -type f -size +1M -delete
echo done
