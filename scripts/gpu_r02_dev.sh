#!/bin/bash
# development (round 2): K1 window 20 / grid 3072 / level-1 pre-test
B="python3 bench.py --steps 200 --warmup 10 --no-secondary --no-cpu-baseline"
scripts/gpu_run.sh r02ae micro 120 tools/micro_k1 z :: \
  pytest 300 python -u -m pytest tests/test_gpu_elements.py tests/test_gpu_configs.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread :: \
  b1 120 $B :: b2 120 $B :: \
  tr 200 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/r02ae/tr -o tr -- python3 bench.py --steps 30 --warmup 3 --no-secondary --no-cpu-baseline
