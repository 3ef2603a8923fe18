set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ingest or file or cli or pcapng or live or host" > $O/tests_r02x.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02x.log)"
timeout -k 10 300 python -u tools/host_inclusive.py --config c2 > $O/host_inclusive_c2.log 2>&1; tail -1 $O/host_inclusive_c2.log
timeout -k 10 300 python -u tools/host_inclusive.py --config c3 > $O/host_inclusive_c3.log 2>&1; tail -1 $O/host_inclusive_c3.log
timeout -k 10 300 python -u tools/live_bench.py --config c2 > $O/live_bench_c2.log 2>&1; tail -1 $O/live_bench_c2.log
