#!/bin/bash
# K1 grid sized for whole windows per wave: micro grid sweep, element parity, bench line
OUT=${OUT:-r03ae}
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  k1o 400 tools/micro_k1o 3 3072 3390 2543 5086 :: \
  tests 600 $T tests/test_gpu_elements.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -k "not c4_full" :: \
  bench 300 python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-secondary
