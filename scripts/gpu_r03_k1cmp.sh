#!/bin/bash
# K1: the micro's back-to-back launches vs the product K1 inside the bench, same box
OUT=${OUT:-r03c}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  k1o 120 tools/micro_k1o 1 :: \
  k1o_trace 120 $P --kernel-trace --stats -d $D/k1o -o k1o -- tools/micro_k1o 1 :: \
  bench 200 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary :: \
  k1o2 120 tools/micro_k1o 1
