#!/bin/bash
# Round 6 (re-entry): the whole GPU suite + smoke on the current tree, then the driver's bench form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06k}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > $O/b20_$i.json 2> $O/b20_$i.err || { tail $O/b20_$i.err; exit 1; }
  cut -c1-300 $O/b20_$i.json
done
B="python3 bench.py --no-cpu-baseline --no-secondary"
for i in 1 2; do
  timeout -k 10 200 $B > $O/ab_main_$i.json 2> $O/ab_main_$i.err || { tail $O/ab_main_$i.err; exit 1; }
  RSV_BENCH_RESOLVE_STREAM=1 timeout -k 10 200 $B > $O/ab_side_$i.json 2> $O/ab_side_$i.err || { tail $O/ab_side_$i.err; exit 1; }
  RSV_BENCH_RESOLVE_STREAM=1 RSV_RESOLVE_SMALL=0 timeout -k 10 200 $B > $O/ab_side1024_$i.json 2> $O/ab_side1024_$i.err || { tail $O/ab_side1024_$i.err; exit 1; }
done
for f in $O/ab_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'], r.get('launches_timed'))"; done
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
echo done
