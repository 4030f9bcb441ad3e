#!/bin/bash
# Round 6: pipeline depth x resolve stream (the forked 256-thread resolve) in the driver's 20-step
# form and at 100 steps; plus the K2 two-deep gather stream-count test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06v}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_segmented.py -k two_deep tests/test_gpu_resolve_stream.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="python3 bench.py --no-cpu-baseline --no-secondary"
for i in 1 2; do
  for cfg in "d2:--depth 2:0" "d3:--depth 3:0" "d3s:--depth 3:1" "d4s:--depth 4:1"; do
    IFS=: read name dflag rs <<< "$cfg"
    RSV_BENCH_RESOLVE_STREAM=$rs timeout -k 10 200 $B $dflag > $O/b_${name}_$i.json 2> $O/b_${name}_$i.err || { tail $O/b_${name}_$i.err; exit 1; }
    RSV_BENCH_RESOLVE_STREAM=$rs timeout -k 10 200 $B $dflag --steps 20 --warmup 5 > $O/b20_${name}_$i.json 2> $O/b20_${name}_$i.err || { tail $O/b20_${name}_$i.err; exit 1; }
  done
done
for f in $O/b*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['steps'], d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'])"; done
echo done
