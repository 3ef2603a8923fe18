#!/bin/bash
# Profile the bench workload on the GPU box (run under gpurun from the repo root).
#   tools/prof.sh <tag> [config]  -> gpurun_out/prof_<tag>/...
# Passes (each its own rocprofv3 run; counters never mixed with runtime traces):
#   1. --kernel-trace --stats           per-kernel durations
#   2. --pmc FETCH_SIZE                 HBM read bytes (gfx950: x2, see MI355X_MICROARCH.md)
#   3. --pmc WRITE_SIZE TCC_EA0_RDREQ_sum
#   4. --pmc SQ_* issue/wait census     (ablations 0,1,2 when PROF_SQ=1)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
TAG=${1:-r01}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/prof_$TAG
mkdir -p "$O"
B=(python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-imix --no-cold --config "$CFG")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- "${B[@]}" > "$O/trace.log" 2>&1
timeout -k 10 240 rocprofv3 --output-format csv --pmc FETCH_SIZE -d "$O/fetch" -o run -- "${B[@]}" > "$O/fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --output-format csv --pmc WRITE_SIZE TCC_EA0_RDREQ_sum -d "$O/write" -o run -- "${B[@]}" > "$O/write.log" 2>&1
if [ "${PROF_SQ:-0}" = "1" ]; then
  for A in 0 1 2; do
    FLUERE_ABLATE=$A timeout -k 10 240 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
      SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$O/sq$A" -o run -- "${B[@]}" > "$O/sq$A.log" 2>&1
    FLUERE_ABLATE=$A timeout -k 10 240 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM \
      SQ_WAIT_INST_LDS -d "$O/lds$A" -o run -- "${B[@]}" > "$O/lds$A.log" 2>&1
  done
fi
python3 "$R/tools/pmc_summary.py" "$O" ${PROF_KERNEL:-} > "$O/summary.txt" 2>&1
# keep the summaries and the kernel-stats tables; drop the bulky per-dispatch CSVs
find "$O" -type f \( -name "*counter_collection.csv" -o -name "*kernel_trace.csv" -o -name "*agent_info.csv" \) -size +1M -delete
du -sh "$O" > "$O/DONE"
