#!/bin/bash
# Round 5: K1's two-group plan vs the grid-stride grid over launch sizes (tools/micro_k1o n)
OUT=${OUT:-r05z2}
exec scripts/gpu_run.sh $OUT \
  sizes 300 tools/micro_k1o n 3e8 4.5e8 6e8 1e9 2e9 4e9 8e9
