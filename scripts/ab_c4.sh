#!/bin/bash
# C4 distinct paths (tools/bench_paths.py) for an A/B of the current build; each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python tools/bench_paths.py --only c4 > gpurun_out/ab_c4_$i.log 2>&1 || exit $?
  python -c "
import json
for l in open('gpurun_out/ab_c4_$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print(d['config'][-40:], round(d['Gelem_s'], 1), d.get('seconds_end_to_end'))"
done
