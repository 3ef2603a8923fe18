#!/bin/bash
# Round 3: the sharded sweep / backward-timestamp / live tests first.
set -eo pipefail
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "sweep or backward or mode_b or tcp_realistic or shard_exchange or sharded or live" > $O/t_sweep.log 2>&1 || { tail -80 $O/t_sweep.log; exit 1; }
tail -3 $O/t_sweep.log
