set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for i in 1 2; do
for f in 1 0; do
RSV_K1_FUSE=$f timeout -k 10 200 python bench.py --steps 400 --warmup 10 --no-cpu-baseline --no-secondary > gpurun_out/ab_$f.log 2>&1 || exit $?
python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$f.log').read().strip().splitlines()[-1]); print('fuse=$f', d['value'], d['ms_per_step'], d['roofline']['launch_avg_us'])"
done; done
