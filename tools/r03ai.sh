#!/bin/bash
# two-phase k_ex_meta + owners at <= 870 flows each: full GPU suite, A/B vs HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03ai; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in tcp c4 c3 tcp tcp_t1; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
