#!/bin/bash
# Round-3 state check (one gpurun call): GPU suite + smoke, default bench line, K1 kernel stats.
OUT=${OUT:-r03a}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  pytest 900 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 500 python3 bench.py :: \
  k1_trace 200 $P --kernel-trace --stats -d $D/k1 -o k1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary
