#!/bin/bash
# Round 5: host heap-replay variants on the GPU box's host CPU (tools/micro_heap2.cpp; no GPU use)
OUT=${OUT:-r05h}
exec scripts/gpu_run.sh $OUT \
  build 120 g++ -O3 -march=native -std=c++17 tools/micro_heap2.cpp -o gpurun_out/$OUT/micro_heap2 :: \
  run 240 gpurun_out/$OUT/micro_heap2 500000000
