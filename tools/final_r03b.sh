#!/bin/bash
# Round-3 closing measurements (second half): GPU suite, smoke, the default
# bench line, every config's bench line, rocprof kernel stats + HBM PMC passes.
#   tools/final_r03b.sh [part1|part2]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final3b
mkdir -p "$O"
cd "$R"
if [ "${1:-part1}" = part1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
  timeout -k 10 300 python -u bench.py > "$O/bench_c2_default.log" 2>&1
  tail -1 "$O/bench_c2_default.log" | cut -c1-300
  for c in c3 c4 c5 c5u tcp tcp_t1 tcp_t1_backtime slow; do
    timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_$c.log" 2>&1
    tail -1 "$O/bench_$c.log" | cut -c1-200
  done
else
  for c in ${2:-c3 c4}; do
    bash tools/prof.sh final3b_$c $c
    cp gpurun_out/prof_final3b_$c/summary.txt "$O/pmc_$c.txt"
  done
fi
