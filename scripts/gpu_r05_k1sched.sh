#!/bin/bash
# Round 5: K1 over static two-group schedules of half windows (W1 waves x A, the rest x B) vs the
# product's 5086-workgroup grid (tools/micro_k1o s)
OUT=${OUT:-r05x3}
exec scripts/gpu_run.sh $OUT \
  sched 300 tools/micro_k1o s 20344:4:4 6144:8:2 6144:10:2 6144:12:1 6144:13:1 6144:8:1 4096:16:1 7168:8:2 5120:12:2 8192:8:2
