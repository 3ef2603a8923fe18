#!/bin/bash
# k_parse_spill PMC (HBM bytes) for c3 / c4 + merge-kernel SQ census (c3)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/final_r03b.sh part2 "c3 c4"
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_r03v_merge; mkdir -p $O
B=(python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --config c3)
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$O/sqa" -o run -- "${B[@]}" > "$O/sqa.log" 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS -d "$O/sqb" -o run -- "${B[@]}" > "$O/sqb.log" 2>&1
python3 $R/tools/pmc_summary.py $O k_merge_partials | tail -3
python3 $R/tools/pmc_summary.py $O k_parse_spill | tail -3
find "$O" -type f -size +1M -delete
