#!/bin/bash
# Round-3 closing measurements (final): smoke, the default bench line (with the
# CPU baseline), every config's bench line, rocprof kernel stats + HBM PMC for c3 / c4 / tcp;
# owner-count probe for C3
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final3c
mkdir -p "$O"
cd "$R"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 300 python -u bench.py > "$O/bench_c2_default.log" 2>&1
tail -1 "$O/bench_c2_default.log" | cut -c1-300
for c in c3 c4 c5 c5u tcp tcp_t1 tcp_t1_backtime slow; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_$c.log" 2>&1
  tail -1 "$O/bench_$c.log" | cut -c1-200
done
for m in 384 512; do
  echo "c3 min owners $m: $(FLUERE_MIN_OWNERS=$m timeout -k 10 200 bash tools/variants.sh 0 c3 base | tail -1)"
done
echo "c3 default: $(timeout -k 10 200 bash tools/variants.sh 0 c3 base | tail -1)"
for c in c3 c4 tcp; do
  bash tools/prof.sh final3c_$c $c
  cp gpurun_out/prof_final3c_$c/summary.txt "$O/pmc_$c.txt"
done
