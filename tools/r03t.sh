#!/bin/bash
# k_parse_spill with the window prefetch: parity, then A/B vs the committed build (variant "r03s")
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03t; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "spill_kernel or full_size" > $O/tests_spill.log 2>&1 || { tail -40 $O/tests_spill.log; exit 1; }
tail -1 $O/tests_spill.log
for c in c3 c4 tcp; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base r03s
done
