#!/bin/bash
# Round 5: ordered distinct over byte keys in one scheduled pass (rsv_wide.hip sample_sched): the wide
# GPU tests (the new pass, the C4 UUID shares incl. hash twins), then the c4w line.
OUT=${OUT:-r05n}
exec scripts/gpu_run.sh $OUT \
  wide 900 python3 -u -m pytest tests/test_gpu_wide_distinct.py tests/test_gpu_wide_keys.py tests/test_gpu_distributed.py -x -q --timeout 600 --timeout-method thread :: \
  c4w 300 python3 tools/bench_paths.py --only c4w
