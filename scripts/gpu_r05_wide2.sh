#!/bin/bash
# Round 5: wide distinct after the set-mode predicted pass: parity, the C4 share lines, kernel stats.
OUT=${OUT:-r05g}
exec scripts/gpu_run.sh $OUT \
  wide 400 python3 -u -m pytest tests/test_gpu_wide_distinct.py -q --timeout 200 --timeout-method thread :: \
  paths 300 python3 tools/bench_paths.py --only c4w :: \
  prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/prof -o c4w -- python3 tools/bench_paths.py --only c4w
