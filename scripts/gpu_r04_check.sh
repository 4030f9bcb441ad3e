#!/bin/bash
# Round 4 end-of-round check on the committed tree: the whole GPU suite, smoke, the default bench line.
OUT=${OUT:-r04e2}
exec scripts/gpu_run.sh $OUT \
  pytest 900 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 600 python3 bench.py
