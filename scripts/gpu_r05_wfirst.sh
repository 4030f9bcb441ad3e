#!/bin/bash
# Round 5: the wide ordered replay through first-occurrence flags: wide GPU tests, then the c4w twins
# line with the flags (default) and without (RSV_FIRST_MIN huge)
OUT=${OUT:-r05u}
exec scripts/gpu_run.sh $OUT \
  wide 900 python3 -u -m pytest tests/test_gpu_wide_distinct.py tests/test_gpu_distributed.py tests/test_gpu_ffm.py -x -q --timeout 600 --timeout-method thread :: \
  c4w 300 python3 tools/bench_paths.py --only c4w :: \
  c4w_set 300 env RSV_FIRST_MIN=1000000000000 python3 tools/bench_paths.py --only c4w
