#!/bin/bash
# Round 5: K1 beside a concurrent 30 us occupier kernel (16 / 64 workgroups), plan vs grid-stride
OUT=${OUT:-r05o}
exec scripts/gpu_run.sh $OUT \
  occ 300 tools/micro_k1o c
