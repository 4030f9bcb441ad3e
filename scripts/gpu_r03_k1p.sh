#!/bin/bash
# K1 pair entries in the product: element parity tests, micro A/B, bench line
OUT=${OUT:-r03u}
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  tests 600 $T tests/test_gpu_elements.py tests/test_gpu_configs.py tests/test_gpu_java_l.py tests/test_gpu_distributed.py tests/test_gpu_wide_keys.py -k "not c4_full" :: \
  k1o 200 tools/micro_k1o 3 3072 :: \
  bench 300 python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary
