#!/bin/bash
# Round 5: K1 window length under the two-group plan (micro_k1o w)
OUT=${OUT:-r05w8}
exec scripts/gpu_run.sh $OUT \
  win 300 tools/micro_k1o w
