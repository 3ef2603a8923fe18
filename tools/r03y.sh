#!/bin/bash
# done-counter grids capped (k_cleanup / k_finalize), no cleanup fence, dynamic merge owners:
# full GPU suite, A/B vs HEAD, 512 minimum owners for C3
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03y; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c4 tcp c3 c2 tcp_t1; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
for m in 512 1024; do
  echo "c3 min owners $m: $(FLUERE_MIN_OWNERS=$m timeout -k 10 200 bash tools/variants.sh 0 c3 base | tail -1)"
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03y c4 tcp
