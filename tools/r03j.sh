#!/bin/bash
# slow-class parity (k_slow paths, fixtures), then the slow bench with kernel stats
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03j; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "middle_path or slow or second_run or spill_overflow or fixture_csv" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for c in slow; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$c -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --config $c > $O/bench_$c.log 2>&1
  f=$(find $O/tr_$c -name "*kernel_stats.csv" | head -1); cp $f $O/ks_$c.csv
  find $O/tr_$c -type f -size +1M -delete
  python3 - $O/ks_$c.csv $c <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:7]:
    n = r["Name"]; n = n[n.find("k_"):][:40] if "k_" in n else n[:40]
    print(sys.argv[2], f'{float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {n}')
PY
  grep metric $O/bench_$c.log | cut -c1-190
done
