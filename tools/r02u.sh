set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
FLUERE_DEBUG=1 timeout -k 10 200 python -u bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg_c2.log 2>&1
grep "\[fluere\]" $O/dbg_c2.log | tail -14
