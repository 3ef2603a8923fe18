set -eo pipefail
cd $GRAFT_REPO_ROOT
for c in c3 c5u c4 tcp; do
  bash tools/prof.sh r02_$c $c
  echo "$c: $(python3 -c "import json; d=json.load(open('gpurun_out/prof_r02_$c/summary.json')); print(d.get('hbm_read_bytes_per_launch'), d.get('hbm_write_bytes_per_launch'))")"
done
