#!/bin/bash
# Round 6: the per-step resolve/publish with write-through (system-scope) result stores and no L2
# write-back before the flag (default) vs the system release (RSV_PUBLISH_WT=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06x}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_elements.py tests/test_gpu_result_take.py tests/test_gpu_resolve_stream.py tests/test_gpu_configs.py tests/test_gpu_host_batch.py -k "not c4" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="python3 bench.py --no-cpu-baseline --no-secondary"
for i in 1 2 3; do
  RSV_PUBLISH_WT=0 timeout -k 10 200 $B > $O/b_wb_$i.json 2> $O/b_wb_$i.err || { tail $O/b_wb_$i.err; exit 1; }
  timeout -k 10 200 $B > $O/b_wt_$i.json 2> $O/b_wt_$i.err || { tail $O/b_wt_$i.err; exit 1; }
done
for i in 1 2; do
  RSV_PUBLISH_WT=0 timeout -k 10 200 $B --steps 20 --warmup 5 > $O/b20_wb_$i.json 2> $O/b20_wb_$i.err || exit 1
  timeout -k 10 200 $B --steps 20 --warmup 5 > $O/b20_wt_$i.json 2> $O/b20_wt_$i.err || exit 1
done
for f in $O/b*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['steps'], d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'])"; done
timeout -k 10 200 rocprofv3 --output-format csv --kernel-trace --stats -d $O/wt -o wt -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary > $O/wt.log 2>&1 || exit 1
grep -h "resolve_publish\|k1_last" $O/wt/wt_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,200-
find $O -name "*_kernel_trace.csv" -delete
echo done
