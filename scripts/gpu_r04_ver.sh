#!/bin/bash
# Round 4: the scheduled merge's verification searches side by side: distinct parity tests, C4 end to
# end, rocprof kernel stats of the ordered path.
OUT=${OUT:-r04v}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  paths 200 python3 tools/bench_paths.py --only c4 :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4o :: \
  trim 30 find $D -name "*_kernel_trace.csv" -delete
