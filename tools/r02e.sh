# kernel-trace stats of the exact engine (tcp, tcp_t1) and the 1M-flow C4 step
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r02e
mkdir -p $O
for c in tcp tcp_t1 c4; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$c -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/$c.log 2>&1
  echo "$c done"
done
find $O -name "*kernel_trace.csv" -size +1M -delete
