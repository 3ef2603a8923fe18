set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests_r02j.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02j.log)"
for c in c2 c3 c4 c5u tcp tcp_t1; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02j_$c.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_r02j_$c.log').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"
done
cd /tmp && export TMPDIR=/tmp
for c in c3 c4 tcp; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_r02j/$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 3 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_r02j_$c.log 2>&1
done
find $GRAFT_REPO_ROOT/$O/prof_r02j -name "*kernel_trace.csv" -size +1M -delete
