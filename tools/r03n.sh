#!/bin/bash
# breakdowns: FLUERE_DEBUG / FLUERE_HOSTPROF clocks (c2, c3, c4), rocprof kernel stats (c4, tcp, tcp_t1), PMC for tcp_t1
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03n; mkdir -p $O
cd $R
for c in c2 c3 c4; do
  FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_$c.log 2>&1
  grep -E "merge phases|per-WG clock|valid|WG starts" $O/dbg_$c.log | tail -4
  FLUERE_HOSTPROF=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 > $O/hp_$c.log 2>&1
  grep "host:" $O/hp_$c.log | tail -3
done
bash tools/r03prof.sh r03n c4 tcp tcp_t1
bash tools/prof.sh r03n_tcp_t1 tcp_t1
cat gpurun_out/prof_r03n_tcp_t1/summary.txt
