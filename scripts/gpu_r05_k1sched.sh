#!/bin/bash
# Round 5: K1 over static two-group schedules of half windows (W1 waves x A, the rest x B) vs the
# product's 5086-workgroup grid (tools/micro_k1o s)
OUT=${OUT:-r05x4}
exec scripts/gpu_run.sh $OUT \
  sched 300 tools/micro_k1o s 6144:10:2 6144:10:3 6144:10:4 6144:11:3 6144:9:3 5120:12:3 6144:11:2 6144:9:2 5632:11:3
