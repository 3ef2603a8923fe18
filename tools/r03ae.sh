#!/bin/bash
# Hot-pass filter words for the exact engine (phash): parity, A/B FLUERE_PHASH=0 vs the prediction
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03ae; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "phash or tcp or fixture or complex or mode_b or rerun" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in tcp tcp tcp_t1 c2; do
  for p in 0 ""; do
    out=$(FLUERE_PHASH=$p timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config $c 2>&1 | grep '^{')
    echo "$c phash=${p:-auto} $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "step_ms", j["ms_per_step"], "recs", j["records"])')"
  done
done
