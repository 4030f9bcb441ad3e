#!/bin/bash
# Round 4: the ordered distinct path with the device-planned scheduled pass (ctl_plan): the ordered
# parity tests, C4 end to end (identity / set / ordered, replay branch) and a kernel trace of the
# ordered C4 share.
OUT=${OUT:-r04f}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -m gpu -q -rfE --timeout 300 --timeout-method thread :: \
  paths 300 python3 tools/bench_paths.py --only c4,c4r,c3k :: \
  c4o_trace 300 $P --kernel-trace --stats -d $D/c4o -o c4o -- python3 tools/bench_paths.py --only c4o
