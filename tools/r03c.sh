#!/bin/bash
# Round 3: full GPU suite, then the bench lines of every config.
set -eo pipefail
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1
tail -1 $O/bench_c2.log | cut -c1-400
for c in c3 c4 tcp tcp_t1 slow c5u; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | cut -c1-300
done
