#!/bin/bash
# one pair min-scan for next eligible / next FIN: parity, A/B vs HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03aj; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "phash or tcp or fixture or sharded or live or complex or backward or mode_b" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in tcp tcp tcp_t1 tcp_t1_backtime; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
