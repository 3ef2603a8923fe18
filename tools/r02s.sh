set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or exchange or sharded or live" > $O/tests_r02s.log 2>&1
echo "tests ok: $(tail -1 $O/tests_r02s.log)"
FLUERE_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_r02s_gloo2.log 2>&1
echo "gloo2: $(tail -1 $O/bench_r02s_gloo2.log | cut -c1-300)"
timeout -k 10 120 python3 tools/shard_step_time.py 8 > $O/shard_step_r02s.log 2>&1 && timeout -k 10 120 python3 tools/shard_step_time.py 2 >> $O/shard_step_r02s.log 2>&1
tail -5 $O/shard_step_r02s.log
