#!/bin/bash
# SQ / LDS counter passes of one bench config, summarised for one kernel
# (one rocprofv3 run per pass):  tools/sq_kernel.sh <tag> <config> <kernel> [VAR=val ...]
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
TAG=$1; CFG=$2; KERN=$3; shift 3
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/sqk_$TAG
mkdir -p "$O"
B=(python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-imix --no-cold --config "$CFG")
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  env "$@" timeout -s KILL 90 rocprofv3 --output-format csv --pmc $P -d "$O/p$i" -o run -- "${B[@]}" > "$O/p$i.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" "$O" "$KERN" > "$O/summary.txt" 2>&1
find "$O" -type f -name "*counter_collection.csv" -size +1M -delete
cat "$O/summary.txt"
