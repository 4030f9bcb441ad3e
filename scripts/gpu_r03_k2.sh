#!/bin/bash
# K2 with the dense head in whole rounds + stream-ordered set_stream: segmented / element parity,
# micro A/B, the C3 line, and the 2-rank rehearsal with the combine on a communication stream
OUT=${OUT:-r03z}
T="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"
exec scripts/gpu_run.sh $OUT \
  tests 600 $T tests/test_gpu_segmented.py tests/test_gpu_configs.py tests/test_gpu_elements.py tests/test_gpu_distributed.py -k "not c4_full" :: \
  k2r 300 tools/micro_k2 r :: \
  c3 200 python3 tools/bench_paths.py --only c3 :: \
  rehearse 500 env RSV_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --c4-steps 2 --no-cpu-baseline
