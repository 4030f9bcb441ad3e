#!/bin/bash
# Round 5: K1 with the workgroup's leftover entries pooled into its last wave -- micro A/B (per-wave
# body, pooled body, the per-wave body without its final rounds), K1 parity tests, the headline bench.
OUT=${OUT:-r05u}
exec scripts/gpu_run.sh $OUT \
  ab 300 tools/micro_k1o p :: \
  test 400 python3 -u -m pytest tests/test_gpu_elements.py tests/test_gpu_configs.py -q -x --timeout 300 --timeout-method thread :: \
  bench 300 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench2 300 python3 bench.py --no-secondary --no-cpu-baseline
