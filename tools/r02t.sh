set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "second_run or slow or fixture or synthetic or raw" > $O/tests_r02t.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02t.log)"
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02t_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
timeout -k 10 300 python -u bench.py --config slow --no-cpu-baseline > $O/bench_r02t_slow.log 2>&1; b slow
FLUERE_SLOW_ABL=1 timeout -k 10 300 python -u bench.py --config slow --no-cpu-baseline > $O/bench_r02t_slowabl1.log 2>&1; b slowabl1
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_r02t_c2.log 2>&1; b c2
