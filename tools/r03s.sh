#!/bin/bash
# k_parse_spill: parity (forced and chosen), then same-box A/B against k_parse_agg on the many-flow configs
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03s; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "spill_kernel" > $O/tests_spill.log 2>&1 || { tail -40 $O/tests_spill.log; exit 1; }
tail -1 $O/tests_spill.log
b() { timeout -k 10 200 python -u bench.py --config $1 --no-cpu-baseline --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['achieved'])"; }
for c in c3 c4 tcp tcp_t1 slow c2; do
  echo "$c agg   $(FLUERE_SPILL_MODE=0 b $c)"
  echo "$c auto  $(b $c)"
done
FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_c3.log 2>&1 || true
grep -E "merge phases|valid" $O/dbg_c3.log | tail -2
bash tools/r03r.sh
