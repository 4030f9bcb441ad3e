#!/bin/bash
# sched_sort: share of the verification-accumulator atomics (RSV_SCHED_AGG=3 skips them; its
# verdict is wrong, so only the kernel durations are read)
OUT=${OUT:-r03j}
P="rocprofv3 --output-format csv --kernel-trace --stats"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  a1 200 $P -d $D/a1 -o a -- python3 tools/bench_paths.py --only c4o :: \
  a3 200 env RSV_SCHED_AGG=3 $P -d $D/a3 -o a -- python3 tools/bench_paths.py --only c4o :: \
  b1 200 $P -d $D/b1 -o a -- python3 tools/bench_paths.py --only c4o
