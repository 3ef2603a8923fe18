#!/bin/bash
# live-mode parity, breakdown (FLUERE_HOSTPROF) and throughput: c2 and realistic TCP, indexed batches or not
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03k; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "live" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c2 tcp; do
  FLUERE_HOSTPROF=1 timeout -k 10 300 python -u tools/live_bench.py --config $c --packets 3000000 --timeout-ms 1000 > $O/live_prof_$c.log 2>&1
  grep "live batch\|ingest 1\|live export" $O/live_prof_$c.log | tail -4
  for ix in 1 0; do
    timeout -k 10 300 python -u tools/live_bench.py --config $c --timeout-ms 1000 --indexed $ix > $O/live_${c}_ix$ix.json 2>&1
    tail -1 $O/live_${c}_ix$ix.json
  done
done
