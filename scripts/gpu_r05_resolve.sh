#!/bin/bash
# Round 5: where resolve_publish's ~5 us go (tools/probe_resolve)
OUT=${OUT:-r05r2}
exec scripts/gpu_run.sh $OUT \
  probe 120 tools/probe_resolve
