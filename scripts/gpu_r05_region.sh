#!/bin/bash
# Round 5: the bench's timed region at K = 20 / 100 with the timing events created up front
OUT=${OUT:-r05g3}
B="python3 bench.py --no-secondary --no-cpu-baseline"
exec scripts/gpu_run.sh $OUT \
  b20 300 $B --steps 20 --warmup 5 :: \
  b100 300 $B --steps 100 --warmup 10 :: \
  b20b 300 $B --steps 20 --warmup 5 :: \
  region 300 python3 tools/probe_region.py
