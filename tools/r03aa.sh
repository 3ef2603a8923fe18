#!/bin/bash
# per-workgroup counters in k_finalize, byte-granular complex-flow filter: GPU suite, A/B vs HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03aa; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in tcp c4 c2 tcp_t1 c3; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03aa tcp
