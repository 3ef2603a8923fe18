#!/bin/bash
# publish without per-workgroup fences, static first owner: full GPU suite, A/B vs HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03z; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c2 c4 tcp c3 c2; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03z c4 tcp
