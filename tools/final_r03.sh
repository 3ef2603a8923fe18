#!/bin/bash
# Round-3 measurements on the GPU box: GPU tests, smoke, the default
# bench line, every config's bench line, rocprof kernel stats + HBM PMC passes.
#   tools/final_r03.sh [part1|part2]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final3
mkdir -p "$O"
cd "$R"
if [ "${1:-part1}" = part1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -1 "$O/smoke.log"
  timeout -k 10 300 python -u bench.py > "$O/bench_c2_default.log" 2>&1
  tail -1 "$O/bench_c2_default.log"
  for c in c3 c4 c5 c5u tcp tcp_t1 slow; do
    timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_$c.log" 2>&1
    tail -1 "$O/bench_$c.log" | cut -c1-200
  done
else
  for c in c2 c3 c4 tcp tcp_t1; do
    bash tools/prof.sh final3_$c $c
    cp gpurun_out/prof_final3_$c/summary.txt "$O/pmc_$c.txt"
  done
fi
