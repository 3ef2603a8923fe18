set -eo pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u bench.py > $O/bench_r02p_default.log 2>&1
tail -1 $O/bench_r02p_default.log
FLUERE_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_r02p_gloo2b.log 2>&1
echo "gloo2: $(tail -1 $O/bench_r02p_gloo2b.log | cut -c1-400)"
for c in c2 c3 c4 c5u tcp slow; do
  bash tools/prof.sh r02p_$c $c
  echo "$c: $(python3 -c "import json; d=json.load(open('gpurun_out/prof_r02p_$c/summary.json')); print(d.get('hbm_read_bytes_per_launch'), d.get('hbm_write_bytes_per_launch'))")"
done
