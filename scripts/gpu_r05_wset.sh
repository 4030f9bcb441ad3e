#!/bin/bash
# Round 5: wide set mode with an analytic first bound (no filling chunk): wide tests + c4w
OUT=${OUT:-r05w}
exec scripts/gpu_run.sh $OUT \
  wide 900 python3 -u -m pytest tests/test_gpu_wide_distinct.py tests/test_gpu_wide_keys.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -x -q --timeout 600 --timeout-method thread :: \
  c4w 300 python3 tools/bench_paths.py --only c4w
