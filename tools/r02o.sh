set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r02o.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02o.log)"
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02o_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
for c in slow c2 c3 tcp; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02o_$c.log 2>&1; b $c
done
FLUERE_HOSTPROF=1 timeout -k 10 120 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline > $O/hostprof_c2.log 2>&1
tail -8 $O/hostprof_c2.log | head -7
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r02o/slow -o run -- python3 $R/bench.py --config slow --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/prof_r02o_slow.log 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $R/$O/prof_r02o_slowpmc/fetch -o run -- python3 $R/bench.py --config slow --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/prof_r02o_slowpmc.log 2>&1
timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $R/$O/prof_r02o_slowpmc/write -o run -- python3 $R/bench.py --config slow --steps 3 --warmup 1 --no-cpu-baseline >> $R/$O/prof_r02o_slowpmc.log 2>&1
python3 $R/tools/pmc_summary.py $R/$O/prof_r02o_slowpmc k_slow | tail -3
find $R/$O -name "*kernel_trace.csv" -size +1M -delete
find $R/$O -name "*counter_collection.csv" -size +2M -delete
