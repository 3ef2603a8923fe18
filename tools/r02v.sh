set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02v_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
for c in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02v_$c.log 2>&1; b $c
done
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_r02v_c2b.log 2>&1; b c2b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "synthetic or fixture or tcp" > $O/tests_r02v.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02v.log)"
