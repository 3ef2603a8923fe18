#!/bin/bash
# lean spill-record path in the merge: parity (spill / many-flow / tcp / sharded), A/B vs HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03w; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "spill or full_size or tcp_realistic or sharded or synthetic or slow or backward or c4_recipe" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c3 c4 tcp; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
