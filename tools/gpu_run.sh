#!/bin/bash
# One GPU-box pass, every GPU step under its own time limit, stopping at the
# first failure:
#   tools/gpu_run.sh <tag> <steps...>
# steps: tests[:<pytest -k expr>]  smoke  bench  cfg:<config>  cold:<config>  prof:<config>
#        trace:<config> (kernel timeline of the last step)  debug:<config> (FLUERE_DEBUG counters)
#        vtrace:<variant>:<config>  hostinc:<config> (host-inclusive rate)  h2d (copy rates)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for st in "$@"; do
  case "$st" in
    tests*)
      K=${st#tests}; K=${K#:}
      if [ -n "$K" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
      fi
      tail -1 "$O/tests.log" ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$O/bench_default.log" 2>&1
      tail -1 "$O/bench_default.log" | cut -c1-400 ;;
    cfg:*)
      c=${st#cfg:}
      timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_$c.log" 2>&1
      tail -1 "$O/bench_$c.log" | cut -c1-300 ;;
    ecfg:*)  # ecfg:<VAR=VALUE>:<config>: cfg with one environment setting (A/B)
      v=${st#ecfg:}; c=${v#*:}; v=${v%%:*}
      env "$v" timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline > "$O/bench_${c}_${v%%=*}.log" 2>&1
      tail -1 "$O/bench_${c}_${v%%=*}.log" | cut -c1-300 ;;
    cold:*)
      c=${st#cold:}
      FLUERE_HOSTPROF=1 timeout -k 10 120 python -u tools/cold_probe.py $c 3 > "$O/cold_$c.log" 2>&1
      grep rep "$O/cold_$c.log" ;;
    prof:*)
      c=${st#prof:}
      bash tools/prof.sh ${TAG}_$c $c
      cp gpurun_out/prof_${TAG}_$c/summary.txt "$O/pmc_$c.txt"
      cp gpurun_out/prof_${TAG}_$c/summary.json "$O/pmc_$c.json"
      f=$(find gpurun_out/prof_${TAG}_$c/trace -name "*kernel_stats.csv" | head -1)
      cp "$f" "$O/kernel_stats_$c.csv" ;;
    trace:*)
      c=${st#trace:}
      bash tools/trace.sh $TAG $c
      cp gpurun_out/trace_${TAG}_$c/timeline.txt "$O/timeline_$c.txt" ;;
    etrace:*)  # etrace:<VAR=VALUE>:<config>: trace with one environment setting (A/B)
      v=${st#etrace:}; c=${v#*:}; v=${v%%:*}
      env "$v" bash tools/trace.sh ${TAG}_e $c
      cp gpurun_out/trace_${TAG}_e_$c/timeline.txt "$O/timeline_${c}_${v%%=*}.txt" ;;
    vtrace:*)  # vtrace:<variant>:<config>: the kernel timeline of a variant build (tools/variants.sh)
      v=${st#vtrace:}; c=${v#*:}; v=${v%%:*}
      FLUERE_LIB=$R/fluere_amd/variants/libfluere_gpu_$v.so bash tools/trace.sh ${v} $c
      cp gpurun_out/trace_${v}_$c/timeline.txt "$O/timeline_${v}_$c.txt" ;;
    hostinc:*)  # hostinc:<config>: fluere offline on a file in the page cache (host-inclusive rate), with host timings
      c=${st#hostinc:}
      FLUERE_HOSTPROF=1 timeout -k 10 300 python -u tools/host_inclusive.py --config $c > "$O/hostinc_$c.log" 2>&1
      tail -3 "$O/hostinc_$c.log" ;;
    h2d)  # host -> HBM copy rate by staging allocation kind
      timeout -k 10 120 ./tools/h2d_probe 4096 32 > "$O/h2d.log" 2>&1
      cat "$O/h2d.log" ;;
    debug:*)
      c=${st#debug:}
      FLUERE_DEBUG=1 timeout -k 10 240 python -u bench.py --config $c --no-cpu-baseline --no-imix --steps 2 --warmup 1 > "$O/debug_$c.log" 2>&1
      grep -E "merge|XCD|WG" "$O/debug_$c.log" | tail -14 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "all done"
