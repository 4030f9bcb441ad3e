#!/bin/bash
# development (round 2): K2 compact FIFO entries / select / draw_j
scripts/gpu_run.sh r02ag pytest 300 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread :: \
  c3a 200 python3 tools/bench_paths.py --only c3 :: c3b 200 python3 tools/bench_paths.py --only c3 :: \
  tr 200 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/r02ag/tr -o tr -- python3 tools/bench_paths.py --only c3
