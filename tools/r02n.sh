set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "synthetic or fixture or tcp or sharded" > $O/tests_r02n.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02n.log)"
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02n_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
for c in c2 tcp c5u; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02n_$c.log 2>&1; b $c
done
FLUERE_HOSTPROF=1 timeout -k 10 120 python -u bench.py --config c2 --steps 8 --warmup 2 --no-cpu-baseline > $O/hostprof_c2.log 2>&1
tail -5 $O/hostprof_c2.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in slow c4; do
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $R/$O/prof_r02n_$c/sq -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/prof_r02n_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc FETCH_SIZE -d $R/$O/prof_r02n_$c/fetch -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline >> $R/$O/prof_r02n_$c.log 2>&1
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc WRITE_SIZE -d $R/$O/prof_r02n_$c/write -o run -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline >> $R/$O/prof_r02n_$c.log 2>&1
done
for k in k_merge_partials k_finalize k_parse_agg k_cleanup; do for c in slow c4; do echo "== $c $k"; python3 $R/tools/pmc_summary.py $R/$O/prof_r02n_$c $k | tail -4; done; done
find $R/$O -name "*counter_collection.csv" -size +2M -delete
