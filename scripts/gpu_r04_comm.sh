#!/bin/bash
# Round 4: the N>1 step's combine on a communication stream: the distributed parity test (2 and 3
# gloo ranks on one GPU) and the 2-rank bench rehearsal.
OUT=${OUT:-r04c2}
exec scripts/gpu_run.sh $OUT \
  tests 400 python3 -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q -rfE --timeout 300 --timeout-method thread :: \
  rehearse 500 env RSV_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --c4-steps 3 --no-cpu-baseline
