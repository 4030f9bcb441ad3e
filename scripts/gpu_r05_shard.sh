#!/bin/bash
# Round 5: the K1 two-group schedule on 8-GPU-like shards (block-unaligned, across index 2^33)
OUT=${OUT:-r05sh}
exec scripts/gpu_run.sh $OUT \
  test 400 python3 -u -m pytest tests/test_gpu_configs.py -k "c2" -v -x --timeout 300 --timeout-method thread
