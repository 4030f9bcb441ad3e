#!/bin/bash
# sched_filter cost split (kernel durations by rocprofv3): product vs log-only vs no candidates
OUT=${OUT:-r03r}
P="rocprofv3 --output-format csv --kernel-trace --stats"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  a1 200 $P -d $D/a1 -o a -- python3 tools/bench_paths.py --only c4o :: \
  v2 200 env RSV_DEV_SCHED_OCC=2 $P -d $D/v2 -o a -- python3 tools/bench_paths.py --only c4o :: \
  v3 200 env RSV_DEV_SCHED_OCC=3 $P -d $D/v3 -o a -- python3 tools/bench_paths.py --only c4o
