set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -k "tcp_10m" > $O/tests_r02d.log 2>&1
echo tests ok
for c in tcp tcp_t1 c4 c3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02d_$c.log 2>&1
  tail -1 $O/bench_r02d_$c.log
done
