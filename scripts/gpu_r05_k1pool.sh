#!/bin/bash
# Round 5: K1 with the workgroup's last rounds pooled -- A/B, the element-path GPU tests, the bench
OUT=${OUT:-r05x}
exec scripts/gpu_run.sh $OUT \
  k1o 200 tools/micro_k1o 3 5086 :: \
  tests 900 python3 -u -m pytest tests/test_gpu_elements.py tests/test_gpu_indexed.py tests/test_gpu_ffm.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_resolve_stream.py -x -q --timeout 600 --timeout-method thread :: \
  bench 300 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench2 300 python3 bench.py --no-secondary --no-cpu-baseline
