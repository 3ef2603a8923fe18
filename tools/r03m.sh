#!/bin/bash
# re-entry check: full GPU suite at HEAD, then the default and C3/C4/tcp bench lines
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03m; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.log 2>&1
tail -1 $O/bench_c2.log | cut -c1-400
for c in c3 c4 tcp; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | cut -c1-300
done
