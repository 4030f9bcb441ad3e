#!/bin/bash
# the whole GPU suite + smoke (what the driver runs at round end)
OUT=${OUT:-r03d}
exec scripts/gpu_run.sh $OUT \
  pytest 900 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
