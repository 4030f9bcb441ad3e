#!/bin/bash
OUT=${OUT:-r03c}
T="python3 -u -m pytest -x -v --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  repro 120 python3 -u tools/dev/repro_merge3.py :: \
  c4share 200 $T --timeout 150 tests/test_gpu_configs.py -k set_mode_identity :: \
  c4full 700 $T tests/test_gpu_configs.py -k c4_full :: \
  rehearse 400 env RSV_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --c4-steps 3
