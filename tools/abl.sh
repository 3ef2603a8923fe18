cd $GRAFT_REPO_ROOT
for A in 1 2 0; do
FLUERE_ABLATE=$A timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl_$A.log 2>&1 || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$A.log').read().strip().splitlines()[-1]); print('abl $A', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
