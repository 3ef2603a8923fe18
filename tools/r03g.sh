#!/bin/bash
# k_slow ablations: 0 full, 1 no dictionary, 2 no parse (diagnostics; wrong results)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for A in 2 3; do
  O=$R/gpurun_out/r03g/abl$A; mkdir -p $O
  FLUERE_SLOW_ABL=$A timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --config slow > $O/trace.log 2>&1
  f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
  find $O/trace -type f -size +1M -delete
  python3 - $O/kernel_stats.csv $A <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    n = r["Name"]; n = n[n.find("k_"):][:40] if "k_" in n else n[:40]
    print(sys.argv[2], f'{float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {n}')
PY
done
