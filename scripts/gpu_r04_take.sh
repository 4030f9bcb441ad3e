#!/bin/bash
# Round 4: result() by buffer hand-over (rsv_result_take): the whole GPU suite, smoke, C4 end to end
# and the host split probe.
OUT=${OUT:-r04t}
exec scripts/gpu_run.sh $OUT \
  pytest 900 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  paths 200 python3 tools/bench_paths.py --only c4 :: \
  probe 200 python3 tools/probe_c4_host.py
