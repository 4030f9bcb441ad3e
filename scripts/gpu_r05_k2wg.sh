#!/bin/bash
# Round 5: K2 workgroup-per-stream form (k >= 512) parity + the large-k line; wide distinct lines.
OUT=${OUT:-r05h}
exec scripts/gpu_run.sh $OUT \
  seg 400 python3 -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_wide_distinct.py -q -x --timeout 200 --timeout-method thread :: \
  paths 400 python3 tools/bench_paths.py --only c3k,c3,c4w :: \
  prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/prof -o c4w -- python3 tools/bench_paths.py --only c3k,c4w
