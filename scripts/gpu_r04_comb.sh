#!/bin/bash
# Round 4: the device combine (C4 merge of 8 shard sets), the index-only C2 path, and the 2-rank
# gloo rehearsal of the N>1 bench's C4 leg (sampling vs combine split); rocprof kernel stats of the merge.
OUT=${OUT:-r04c}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  paths 300 python3 tools/bench_paths.py --only c4m,c2i :: \
  c4m_trace 300 $P --kernel-trace --stats -d $D/c4m -o c4m -- python3 tools/bench_paths.py --only c4m :: \
  rehearse 500 env RSV_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --c4-steps 3 --no-cpu-baseline
