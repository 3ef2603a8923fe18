#!/bin/bash
# host-side A/B on one box: stream-query rate in the poll loops, mailbox vs copy+sync
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03r; mkdir -p $O
cd $R
b() { timeout -k 10 200 python -u bench.py --config $1 --no-cpu-baseline --steps ${2:-20} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"; }
for rep in 1 2; do
  echo "c2 mask65535 $(b c2 40)"; echo "c2 mask1023 $(FLUERE_QUERY_MASK=1023 b c2 40)"
  echo "tcp mail $(b tcp)"; echo "tcp nomail $(FLUERE_NO_MAIL=1 b tcp)"
  echo "tcp_t1 mail $(b tcp_t1)"; echo "tcp_t1 nomail $(FLUERE_NO_MAIL=1 b tcp_t1)"
done
