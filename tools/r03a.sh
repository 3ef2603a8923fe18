set -eo pipefail
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c2.log 2>&1
tail -1 $O/bench_c2.log
for c in c3 c4 tcp tcp_t1 slow c5u; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.log 2>&1
  tail -1 $O/bench_$c.log | cut -c1-300
done
