#!/bin/bash
# Round 5: K1 with dynamic half-window claims (persistent waves) vs the product's oversubscribed grid
OUT=${OUT:-r05v}
exec scripts/gpu_run.sh $OUT \
  dyn 300 tools/micro_k1o y
