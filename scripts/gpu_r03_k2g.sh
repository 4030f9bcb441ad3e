#!/bin/bash
# K2 at up to 128 workgroups per CU with the 32-bit threshold table: segmented parity, the C3 full
# launch, a grid sweep, the C3 line
OUT=${OUT:-r03aj}
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  tests 600 $T tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "segmented or ragged or fifo or c3 or stream or large" :: \
  k2g 400 tools/micro_k2 G 4096 16384 32768 65536 :: \
  c3 200 python3 tools/bench_paths.py --only c3
