#!/bin/bash
# Round 4: sched_bin_sort on one-register fine buckets only (larger ones listed for sched_big_sort),
# 2048-entry bins: distinct parity tests, C4 end to end, kernel stats, and the big-bucket count on
# the hash-twin stream (RSV_SCHED_DEBUG).
OUT=${OUT:-r04b2}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  paths 200 python3 tools/bench_paths.py --only c4 :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4o :: \
  twins 200 env RSV_SCHED_DEBUG=1 python3 tools/bench_paths.py --only c4r :: \
  trim 30 find $D -name "*_kernel_trace.csv" -delete
