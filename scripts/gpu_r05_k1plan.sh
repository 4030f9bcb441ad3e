#!/bin/bash
# Round 5: K1's two-group schedule in the product -- K1 parity tests, then the headline bench A/B/A/B
# against the previous build (reservoir_amd/libreservoir_hip_base.so, grid-stride K1)
OUT=${OUT:-r05y}
A="bench.py --no-secondary --no-cpu-baseline"
B="python3 $A"
exec scripts/gpu_run.sh $OUT \
  base1 300 python3 tools/with_lib.py reservoir_amd/libreservoir_hip_base.so $A :: \
  new1 300 $B :: \
  base2 300 python3 tools/with_lib.py reservoir_amd/libreservoir_hip_base.so $A :: \
  new2 300 $B
