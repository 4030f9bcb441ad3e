#!/bin/bash
# development (round 2): K2 512-entry FIFO + overflow rounds
scripts/gpu_run.sh r02ak pytest 300 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread :: \
  q 120 tools/micro_k2 q :: \
  tr 200 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/r02ak/tr -o tr -- python3 tools/bench_paths.py --only c3
