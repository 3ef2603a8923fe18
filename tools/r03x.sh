#!/bin/bash
# bulk table clears (many-flow runs): parity, A/B vs HEAD; merge record-phase spread (C3, C4)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03x; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "spill or rerun or tcp_realistic or sharded or c4_recipe or file or live" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c4 tcp c3; do
  timeout -k 10 300 bash tools/variants.sh "0" $c base head
done
for c in c3 c4; do
  FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_$c.log 2>&1 || true
  grep -E "record phase per|merge phases" $O/dbg_$c.log | tail -2
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03x c4
