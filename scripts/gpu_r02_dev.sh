#!/bin/bash
# development (round 2): distinct/config GPU tests, C4 timings
D=gpurun_out/r02t
scripts/gpu_run.sh r02t tests 500 python -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py -m gpu -x -q -rfE --timeout 200 --timeout-method thread :: \
  c4 200 env RSV_SCHED_DEBUG=1 python3 tools/bench_paths.py --only c4,c4r
