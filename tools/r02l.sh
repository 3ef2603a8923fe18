set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "synthetic or generator or sharded or mac or raw or live" > $O/tests_r02l.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02l.log)"
for c in slow c3 c5u c4 c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02l_$c.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('$O/bench_r02l_$c.log').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"
done
for c in c3 slow; do bash tools/prof.sh r02l_$c $c; echo "$c: $(python3 -c "import json; d=json.load(open('gpurun_out/prof_r02l_$c/summary.json')); print(d.get('hbm_read_bytes_per_launch'), d.get('hbm_write_bytes_per_launch'))")"; done
