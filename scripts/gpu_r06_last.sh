#!/bin/bash
# Round 6, last tree: the whole GPU suite, smoke, the driver's bench form and the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06L}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for f in $O/bench20.json $O/bench.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['steps'], d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'], r['launches_timed'])"; done
for i in 1 2; do
  RSV_REPLAY_DEBUG=1 timeout -k 10 300 python3 tools/bench_paths.py --only c4r > $O/c4r_$i.log 2>&1 || exit 1
done
grep -h "rsv replay" $O/c4r_1.log | tail -3
grep -h '^{' $O/c4r_*.log | python3 -c "import json,sys; [print('c4r', json.loads(l)['seconds_end_to_end']) for l in sys.stdin]"
echo done
