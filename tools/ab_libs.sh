#!/bin/bash
# Same-box A/B of library builds and environment settings on one bench config
# (diagnostics):  tools/ab_libs.sh <config> <reps> "<lib>:<VAR=VAL>" ...
#   lib: "base" (the in-tree library) or a name under fluere_amd/variants/
#   (libfluere_gpu_<name>.so); VAR=VAL: one environment setting ("-" for none)
R=${GRAFT_REPO_ROOT:-/root/repo}
CFG=$1; REPS=$2; shift 2
for rep in $(seq 1 "$REPS"); do
  for spec in "$@"; do
    l=${spec%%:*}; e=${spec#*:}
    if [ "$l" = base ]; then LIB=""; else LIB="$R/fluere_amd/variants/libfluere_gpu_$l.so"; fi
    [ "$e" = "-" ] && e="FLUERE_AB_NONE=1"
    out=$(env "$e" FLUERE_LIB=$LIB timeout -k 10 120 python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-imix --no-cold --config "$CFG" 2>&1 | grep '^{') || { echo "$spec FAILED"; exit 1; }
    echo "rep $rep $spec $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "step_ms", j["ms_per_step"], "recs", j["records"])')"
  done
done
