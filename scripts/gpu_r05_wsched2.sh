#!/bin/bash
OUT=${OUT:-r05o}
exec scripts/gpu_run.sh $OUT \
  c4w 300 env RSV_WIDE_SCHED_DEBUG=1 python3 tools/bench_paths.py --only c4w :: \
  c4w0 300 env RSV_WIDE_SCHED=0 python3 tools/bench_paths.py --only c4w :: \
  wide 900 python3 -u -m pytest tests/test_gpu_wide_distinct.py -x -q --timeout 600 --timeout-method thread
