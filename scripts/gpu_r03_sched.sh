#!/bin/bash
# ordered distinct with the bucket filing split out of the pass: parity + timing + kernel stats
OUT=${OUT:-r03s}
P="rocprofv3 --output-format csv --kernel-trace --stats"
D=gpurun_out/$OUT
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  tests 600 $T tests/test_gpu_distinct.py tests/test_gpu_configs.py -k "distinct or c4_share or ordered" :: \
  c4o 200 python3 tools/bench_paths.py --only c4,c4r :: \
  prof 200 $P -d $D/p -o a -- python3 tools/bench_paths.py --only c4o
