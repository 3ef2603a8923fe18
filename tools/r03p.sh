#!/bin/bash
# spill-store question (ABL 4: coalesced raw append instead of owner segments), merge record loop U = 1/2/4, slow config
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03p; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "slow or general or full_size or tcp_realistic or sharded" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c3 c4; do
  for a in 0 4; do
    FLUERE_ABLATE=$a FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_${c}_$a.log 2>&1 || true
    echo "$c abl $a"; grep -E "XCD 0: WG|per-WG clock|merge phases" $O/dbg_${c}_$a.log | tail -3
  done
  timeout -k 10 600 bash tools/variants.sh "0 4" $c base mu2 mu4
done
timeout -k 10 300 bash tools/variants.sh "0" tcp base mu4
timeout -k 10 200 python -u bench.py --config slow --no-cpu-baseline > $O/bench_slow.log 2>&1
tail -1 $O/bench_slow.log | cut -c1-250
