#!/bin/bash
# Round 4: sched_bin_file workgroup size A/B (dev builds: 512 / 256 threads, 4 entries each):
# rocprof kernel stats of the ordered path.
OUT=${OUT:-r04f2}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4o :: \
  f512 200 $P --kernel-trace --stats -d $D/f512 -o f512 -- $W reservoir_amd/libreservoir_hip_expf512.so tools/bench_paths.py --only c4o :: \
  f256 200 $P --kernel-trace --stats -d $D/f256 -o f256 -- $W reservoir_amd/libreservoir_hip_expf256.so tools/bench_paths.py --only c4o :: \
  trim 30 find $D -name "*_kernel_trace.csv" -delete
