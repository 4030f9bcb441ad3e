#!/bin/bash
# Round 5: the bench's samplers in flight, A/B/A/B (2 / 3 / 4)
OUT=${OUT:-r05d2}
B="python3 bench.py --no-secondary --no-cpu-baseline"
exec scripts/gpu_run.sh $OUT \
  d2 300 $B --depth 2 :: d3 300 $B --depth 3 :: d4 300 $B --depth 4 :: \
  d2b 300 $B --depth 2 :: d3b 300 $B --depth 3 :: d4b 300 $B --depth 4
