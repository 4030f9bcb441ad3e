#!/bin/bash
# Round 5 closing run: the whole GPU suite, smoke, the default bench line
OUT=${OUT:-r05L4}
exec scripts/gpu_run.sh $OUT \
  gpu 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 600 python3 bench.py --steps 20 --warmup 5
