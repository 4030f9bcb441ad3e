#!/bin/bash
# Round 6: K1 step overhead -- the two-dispatch step (K1, then the one-workgroup resolve/publish) vs
# the fused kernel (RSV_K1_FUSE=1), alternating; a kernel trace of the default step; the byte-key
# merge with wb_prep (tests + c4w)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06j}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide_distinct.py tests/test_gpu_wide_keys.py tests/test_gpu_elements.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="python3 bench.py --no-cpu-baseline --no-secondary"
for i in 1 2; do
  timeout -k 10 200 $B > $O/b_two_$i.json 2> $O/b_two_$i.err || { tail $O/b_two_$i.err; exit 1; }
  RSV_K1_FUSE=1 timeout -k 10 200 $B > $O/b_fused_$i.json 2> $O/b_fused_$i.err || { tail $O/b_fused_$i.err; exit 1; }
done
for f in $O/b_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'], r.get('launches_timed'))"; done
P="rocprofv3 --output-format csv --kernel-trace"
timeout -k 10 200 $P -d $O/bt -o bt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 > $O/bt.log 2>&1 || exit $?
python3 tools/trace_window.py $O/bt/bt_kernel_trace.csv k1_last_writer 45 > $O/bt_timeline.txt || exit $?
find $O -name "*_kernel_trace.csv" -delete
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_paths.py --only c4w > $O/w_bucket_$i.log 2>&1 || exit $?
done
grep -h '^{' $O/w_*.log | cut -c1-250
echo done
