#!/bin/bash
# Round 6: the N > 1 bench path rehearsed with 2 and 4 gloo ranks sharing one GPU (the 8-GPU RCCL
# run is the driver's), plus the RCCL world-1 child-process test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06y}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_distributed.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
RSV_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --c4-steps 3 --no-cpu-baseline > $O/rehearse2.log 2>&1 || { tail -20 $O/rehearse2.log; exit 1; }
grep -h '^{' $O/rehearse2.log | cut -c1-400
RSV_BENCH_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 10 --warmup 2 --c4-steps 2 --no-cpu-baseline --no-secondary > $O/rehearse4.log 2>&1 || { tail -20 $O/rehearse4.log; exit 1; }
grep -h '^{' $O/rehearse4.log | cut -c1-400
echo done
