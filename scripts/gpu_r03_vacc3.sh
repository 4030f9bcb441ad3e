#!/bin/bash
# GPU suite + smoke on the final tree, then the accumulator-atomics A/B (RSV_SCHED_AGG=3 skips
# them; only kernel durations are read)
OUT=${OUT:-r03l}
P="rocprofv3 --output-format csv --kernel-trace --stats"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  pytest 900 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  a1 200 $P -d $D/a1 -o a -- python3 tools/bench_paths.py --only c4o :: \
  a3 200 env RSV_SCHED_AGG=3 $P -d $D/a3 -o a -- python3 tools/bench_paths.py --only c4o
