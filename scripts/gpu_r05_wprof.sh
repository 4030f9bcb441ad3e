#!/bin/bash
# Round 5: kernel trace of the C4 UUID ordered share (scheduled pass) for its timeline
OUT=${OUT:-r05p}
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  trace 300 rocprofv3 --output-format csv --kernel-trace --stats -d $D/w -o w -- python3 tools/bench_paths.py --only c4w :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +12M -delete
