set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ingest or file or cli or pcapng or live" > $O/tests_r02y.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02y.log)"
for cfg in c3 c2; do
for mode in kernel sdma; do
  FLUERE_HOSTPROF=1 FLUERE_INGEST_COPY=$mode timeout -k 10 300 python -u tools/host_inclusive.py --config $cfg --reps 2 > $O/hi_${cfg}_$mode.log 2>&1
  echo "$cfg $mode: $(tail -1 $O/hi_${cfg}_$mode.log | cut -c1-330)"
  grep "ingest" $O/hi_${cfg}_$mode.log | tail -1
done
done
