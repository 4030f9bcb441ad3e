#!/bin/bash
# Round 5: the whole GPU suite + smoke on the current tree
OUT=${OUT:-r05s}
exec scripts/gpu_run.sh $OUT \
  gpu 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
