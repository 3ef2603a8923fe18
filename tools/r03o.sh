#!/bin/bash
# exact engine: mailbox reads, Mode B records with order words; k_finalize with the register parser + deferral
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03o; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c2 c3 c4 tcp tcp_t1 slow; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
for a in 1 2; do
  FLUERE_CLEAN_ABL=$a timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline --steps 10 > $O/abl_c4_$a.log 2>&1 || true
  tail -1 $O/abl_c4_$a.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03o tcp tcp_t1 c4
