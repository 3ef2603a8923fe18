#!/bin/bash
# SQ counter passes for k_parse_agg on a bench config (one rocprofv3 run per
# pass; counters never mixed with runtime traces).
#   tools/sq_prof.sh <tag> "<ablations>" [config]  -> gpurun_out/sq_<tag>/...
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
TAG=${1:-x}
ABLS=${2:-0}
CFG=${3:-c2}
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/sq_$TAG
mkdir -p "$O"
B=(python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --config "$CFG")
P1="SQ_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY"
P2="SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_BRANCH"
P3="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM"
P4="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_ATOMIC SQ_INST_LEVEL_LDS SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT64"
for A in $ABLS; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    FLUERE_ABLATE=$A timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P -d "$O/a${A}p$i" -o run -- "${B[@]}" > "$O/a${A}p$i.log" 2>&1
  done
done
python3 "$R/tools/pmc_summary.py" "$O" > "$O/summary.txt" 2>&1
find "$O" -type f \( -name "*counter_collection.csv" \) -size +1M -delete
cat "$O/summary.txt"
