#!/bin/bash
# Round 5: the bench with the first timed launch moved off the region's first step, 20 and 100 steps
OUT=${OUT:-r05b2}
B="python3 bench.py --no-secondary --no-cpu-baseline"
exec scripts/gpu_run.sh $OUT \
  b20 300 $B --steps 20 --warmup 5 :: \
  b100 300 $B --steps 100 --warmup 10 :: \
  b20b 300 $B --steps 20 --warmup 5 :: \
  b100b 300 $B --steps 100 --warmup 10
