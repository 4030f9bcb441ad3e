#!/bin/bash
# K3 / scheduled-pass grid sweep (RSV_DEV_FGRID), C4 share: filter times by HIP events
OUT=${OUT:-r03ak}
B="python3 tools/bench_paths.py --only c4i,c4o"
exec scripts/gpu_run.sh $OUT \
  g8192 200 env RSV_DEV_FGRID=8192 $B :: \
  g4096 200 env RSV_DEV_FGRID=4096 $B :: \
  g16384 200 env RSV_DEV_FGRID=16384 $B :: \
  g32768 200 env RSV_DEV_FGRID=32768 $B :: \
  g6144 200 env RSV_DEV_FGRID=6144 $B :: \
  g8192b 200 env RSV_DEV_FGRID=8192 $B
