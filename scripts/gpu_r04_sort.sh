#!/bin/bash
# Round 4: the bucketed merges by coarse bins (sched_bin_* for the scheduled pass, set_bin_* for the
# filter path) vs the per-entry filing + one wave per bucket (dev build -DRSV_SCHED_FINE): distinct
# parity tests, C4 end to end (identity / set / ordered) on both builds, rocprof kernel stats.
OUT=${OUT:-r04i}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  paths 200 python3 tools/bench_paths.py --only c4 :: \
  paths_fine 200 $W reservoir_amd/libreservoir_hip_expfine.so tools/bench_paths.py --only c4 :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4 :: \
  fine 200 $P --kernel-trace --stats -d $D/fine -o fine -- $W reservoir_amd/libreservoir_hip_expfine.so tools/bench_paths.py --only c4
