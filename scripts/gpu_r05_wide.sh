#!/bin/bash
# Round 5: K2 after the variant strip (segmented tests), the wide-key C4 share measured, its kernels.
OUT=${OUT:-r05e}
exec scripts/gpu_run.sh $OUT \
  seg 300 python3 -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "segmented or c3" -q --timeout 200 --timeout-method thread :: \
  paths 400 python3 tools/bench_paths.py --only c4w,c3 :: \
  prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/prof -o c4w -- python3 tools/bench_paths.py --only c4w
