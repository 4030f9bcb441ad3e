#!/bin/bash
# Round 4: bin reservations spread over 8 counter copies vs one (dev build -DRSV_BIN_COPIES=1):
# distinct parity tests on the product, rocprof kernel stats of the ordered path on both.
OUT=${OUT:-r04y}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  ks 200 $P --kernel-trace --stats -d $D/ks -o ks -- python3 tools/bench_paths.py --only c4o :: \
  c1 200 $P --kernel-trace --stats -d $D/c1 -o c1 -- $W reservoir_amd/libreservoir_hip_expc1.so tools/bench_paths.py --only c4o :: \
  trim 30 find $D -name "*_kernel_trace.csv" -delete
