#!/bin/bash
# block-compacted k_ex_meta: full GPU suite, then the exact-engine configs and C2/C3/C4
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03q; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in tcp tcp_t1 tcp_t1_backtime c2 c3 c4 slow; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['ms_per_step'], d['roofline']['kernel_ms'], d['sequential_mode'], d['exact_passes'])"
done
cd /tmp && export TMPDIR=/tmp
bash $R/tools/r03prof.sh r03q tcp tcp_t1
cd $R
for c in c3 c4; do
  for a in 0 5 4; do
    FLUERE_ABLATE=$a FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 2 > $O/dbg_${c}_$a.log 2>&1 || true
    echo "$c abl $a"; grep -E "XCD [0-7]: WG" $O/dbg_${c}_$a.log | tail -8 | awk '{print $NF, $(NF-5), $(NF-2)}' | tr '\n' ' '; echo
  done
done
