set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_r02m.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02m.log)"
b() { python3 -c "import json,sys; d=json.loads(open('$O/bench_r02m_$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'], d['records'])"; }
for c in c2 slow c3 c5u c4 tcp; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_r02m_$c.log 2>&1; b $c
done
FLUERE_NO_FUSE=1 timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_r02m_c2nofuse.log 2>&1; b c2nofuse
for A in 1 2; do FLUERE_SLOW_ABL=$A timeout -k 10 300 python -u bench.py --config slow --no-cpu-baseline > $O/bench_r02m_slowabl$A.log 2>&1; b slowabl$A; done
cd /tmp && export TMPDIR=/tmp
for c in c2 slow; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_r02m/$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_r02m_$c.log 2>&1
done
find $GRAFT_REPO_ROOT/$O/prof_r02m -name "*kernel_trace.csv" -size +1M -delete
