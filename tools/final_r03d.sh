#!/bin/bash
# Round-3 closing measurements (last build): full GPU suite, smoke, the default
# bench line (with the CPU baseline), every config's bench line, rocprof kernel
# stats + HBM PMC for c2 / c3 / c4 / tcp / tcp_t1, the realistic-TCP step timeline
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final3d
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 300 python -u bench.py > "$O/bench_c2_default.log" 2>&1
tail -1 "$O/bench_c2_default.log" | cut -c1-300
for c in c3 c4 c5 c5u tcp tcp_t1 tcp_t1_backtime slow; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_$c.log" 2>&1
  tail -1 "$O/bench_$c.log" | cut -c1-200
done
for c in c2 c3 c4 tcp tcp_t1; do
  bash tools/prof.sh final3d_$c $c
  cp gpurun_out/prof_final3d_$c/summary.txt "$O/pmc_$c.txt"
  f=$(find gpurun_out/prof_final3d_$c/trace -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/kernel_stats_$c.csv"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_tcp" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --config tcp > "$O/tr_tcp.log" 2>&1
f=$(find "$O/tr_tcp" -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline_last.py "$f" k_parse > $O/timeline_tcp.txt
find "$O/tr_tcp" -type f -size +1M -delete
tail -1 $O/timeline_tcp.txt
