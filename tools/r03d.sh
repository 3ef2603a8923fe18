#!/bin/bash
# Round 3: exact-engine tests, then tcp / tcp_t1 bench lines and kernel stats.
set -eo pipefail
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "sweep or backward or mode_b or tcp or shard or live or fixture_csv or synthetic" > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -1 $O/t.log
bash tools/r03prof.sh d tcp tcp_t1 tcp_t1_backtime
