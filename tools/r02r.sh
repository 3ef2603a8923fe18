set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r02r.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02r.log)"
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02r_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
for c in c3 c2 c4 c5u tcp; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02r_$c.log 2>&1; b $c
done
FLUERE_SLOW_ABL=1 timeout -k 10 300 python -u bench.py --config slow --no-cpu-baseline > $O/bench_r02r_slowabl1.log 2>&1; b slowabl1
bash tools/prof.sh r02r_c3 c3; echo "c3: $(python3 -c "import json; d=json.load(open('gpurun_out/prof_r02r_c3/summary.json')); print(d.get('hbm_read_bytes_per_launch'), d.get('hbm_write_bytes_per_launch'))")"
