#!/bin/bash
# Round 5: K1 with direct appends (k1_body_q): A/B against the round-4 body, the GPU suite, the bench.
OUT=${OUT:-r05l}
exec scripts/gpu_run.sh $OUT \
  k1o 200 tools/micro_k1o 3 5086 :: \
  gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread :: \
  bench 300 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench2 300 python3 bench.py --no-secondary --no-cpu-baseline
