set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests_r02g.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02g.log)"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r02g.log 2>&1
echo smoke ok
timeout -k 10 300 python -u bench.py > $O/bench_r02g.log 2>&1
tail -1 $O/bench_r02g.log
FLUERE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --config c4 > $O/bench_r02g_dist2.log 2>&1
tail -1 $O/bench_r02g_dist2.log
