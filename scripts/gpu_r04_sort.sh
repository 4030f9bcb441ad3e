#!/bin/bash
# Round 4: ordered path with the deferred zeroing; sched_sort A/B (dev builds: no verification
# atomics / 4 / 16 buckets per wave) by rocprof kernel stats; one SQ counter pass on the product.
OUT=${OUT:-r04i}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -q -rfE --timeout 300 --timeout-method thread :: \
  paths 200 python3 tools/bench_paths.py --only c4o :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4o :: \
  nv 200 $P --kernel-trace --stats -d $D/nv -o nv -- $W reservoir_amd/libreservoir_hip_expnv.so tools/bench_paths.py --only c4o :: \
  b4 200 $P --kernel-trace --stats -d $D/b4 -o b4 -- $W reservoir_amd/libreservoir_hip_expb4.so tools/bench_paths.py --only c4o :: \
  b16 200 $P --kernel-trace --stats -d $D/b16 -o b16 -- $W reservoir_amd/libreservoir_hip_expb16.so tools/bench_paths.py --only c4o :: \
  pmc 120 $P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $D/pmc -o pmc -- python3 tools/bench_paths.py --only c4o
