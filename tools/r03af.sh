#!/bin/bash
# phash A/B (FLUERE_PHASH=0 vs the prediction) and the realistic-TCP timeline with it
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03af; mkdir -p $O
cd $R
for c in tcp tcp tcp_t1 c2; do
  for p in 0 auto; do
    if [ $p = auto ]; then unset FLUERE_PHASH; else export FLUERE_PHASH=$p; fi
    out=$(timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config $c 2>&1 | grep '^{')
    echo "$c phash=$p $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "step_ms", j["ms_per_step"], "recs", j["records"])')"
  done
done
unset FLUERE_PHASH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_tcp" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --config tcp > "$O/tcp.log" 2>&1
f=$(find "$O/tr_tcp" -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline_last.py "$f" k_parse > $O/timeline_tcp.txt
find "$O/tr_tcp" -type f -size +1M -delete
head -20 $O/timeline_tcp.txt; tail -1 $O/timeline_tcp.txt
