#!/bin/bash
# Round 4: replay through first-occurrence flags -- distinct + config parity, the replay line.
OUT=${OUT:-r04fo}
exec scripts/gpu_run.sh $OUT \
  dist 600 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py -q -rfE -x --timeout 300 --timeout-method thread :: \
  twins 300 python3 tools/bench_paths.py --only c4r :: \
  twins_set 300 env RSV_FIRST_MIN=1000000000 python3 tools/bench_paths.py --only c4r
