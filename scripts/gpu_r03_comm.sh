#!/bin/bash
# 2-rank gloo rehearsal A/B: combine on a communication stream (default) vs on the sampling stream
OUT=${OUT:-r03aa}
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --no-c4 --no-cpu-baseline"
exec scripts/gpu_run.sh $OUT \
  off 300 env RSV_BENCH_BACKEND=gloo RSV_BENCH_COMM=0 $R :: \
  on 300 env RSV_BENCH_BACKEND=gloo $R :: \
  off2 300 env RSV_BENCH_BACKEND=gloo RSV_BENCH_COMM=0 $R
