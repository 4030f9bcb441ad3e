#!/bin/bash
# Round 4: packed-key wave sort (one 64-bit word per lane) in every bucketed merge; A/B of the merge
# forms: product (scheduled pass by coarse bins, filter path per bucket), dev builds fine (both per
# bucket) and setbins (both by bins).  Distinct parity tests on the product, C4 end to end and
# rocprof kernel stats on all three.
OUT=${OUT:-r04j}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  paths 200 python3 tools/bench_paths.py --only c4 :: \
  paths_fine 200 $W reservoir_amd/libreservoir_hip_expfine.so tools/bench_paths.py --only c4 :: \
  paths_setbins 200 $W reservoir_amd/libreservoir_hip_expsetbins.so tools/bench_paths.py --only c4 :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4 :: \
  fine 200 $P --kernel-trace --stats -d $D/fine -o fine -- $W reservoir_amd/libreservoir_hip_expfine.so tools/bench_paths.py --only c4 :: \
  setbins 200 $P --kernel-trace --stats -d $D/setbins -o setbins -- $W reservoir_amd/libreservoir_hip_expsetbins.so tools/bench_paths.py --only c4 :: \
  trim 30 find $D -name "*_kernel_trace.csv" -delete
