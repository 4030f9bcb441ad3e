#!/bin/bash
# Round 5: cost of K1's final partial resolve rounds (micro_k1o t: with / without them, grids 5086/1536/3072)
OUT=${OUT:-r05t}
exec scripts/gpu_run.sh $OUT \
  tail 300 tools/micro_k1o t
