#!/bin/bash
# merge-kernel phase clocks (FLUERE_DEBUG) for the many-flow configs
set -eo pipefail
O=gpurun_out/r03f; mkdir -p $O
for c in c3 c4 tcp; do
  FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_$c.log 2>&1
  grep -E "merge phases|per-WG clock|valid" $O/dbg_$c.log | tail -4
done
