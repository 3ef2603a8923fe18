#!/bin/bash
# Time k_parse_agg variants on a bench config (diagnostics).
#   tools/variants.sh "<abls>" [config] [lib names...]
# lib names: builds under fluere_amd/variants/libfluere_gpu_<name>.so ("base" =
# the in-tree library).
R=${GRAFT_REPO_ROOT:-/root/repo}
ABLS=${1:-0}
CFG=${2:-c2}
shift 2 2>/dev/null
LIBS=${*:-base}
for l in $LIBS; do
  if [ "$l" = base ]; then LIB=""; else LIB="$R/fluere_amd/variants/libfluere_gpu_$l.so"; fi
  for a in $ABLS; do
    out=$(FLUERE_LIB=$LIB FLUERE_ABLATE=$a timeout -k 10 120 python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --config "$CFG" 2>&1 | grep '^{') || { echo "lib=$l abl=$a FAILED"; exit 1; }
    echo "lib=$l abl=$a $(echo "$out" | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("kernel_ms", j["roofline"]["kernel_ms"], "GB/s", j["roofline"]["achieved"], "step_ms", j["ms_per_step"], "recs", j["records"])')"
  done
done
