#!/bin/bash
# sched_file cost split (kernel durations): product vs atomics only vs atomics + one store
OUT=${OUT:-r03v}
P="rocprofv3 --output-format csv --kernel-trace --stats"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  a 200 $P -d $D/a -o a -- python3 tools/bench_paths.py --only c4o :: \
  f1 200 env RSV_DEV_FILE=1 $P -d $D/f1 -o a -- python3 tools/bench_paths.py --only c4o :: \
  f2 200 env RSV_DEV_FILE=2 $P -d $D/f2 -o a -- python3 tools/bench_paths.py --only c4o
