#!/bin/bash
# Round 5: K2 two-deep deferred winner gather (asm-issued loads, scalar offsets loads) -- A/B against
# the round-4 kernel (micro_k2 n), the segmented parity tests and the C3 line.
OUT=${OUT:-r05n}
exec scripts/gpu_run.sh $OUT \
  ab 300 tools/micro_k2 n :: \
  seg 600 python3 -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "segmented or c3 or ragged or fifo or long or pow27 or int32 or single" -x -q --timeout 300 --timeout-method thread :: \
  c3 200 python3 tools/bench_paths.py --only c3 :: \
  c3b 200 python3 tools/bench_paths.py --only c3
