#!/bin/bash
set -eo pipefail
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "sweep or backward or mode_b or tcp or shard or live or fixture or synthetic" > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -1 $O/t.log
for c in tcp tcp_t1 tcp_t1_backtime; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | cut -c1-250
done
bash tools/r03prof.sh e tcp_t1
