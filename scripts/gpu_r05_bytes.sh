#!/bin/bash
# Round 5: the byte basis of random 8-B gathers (tools/micro_gather line probes): time, then the
# L2's memory-side read requests and FETCH_SIZE per probe, each counter set in its own pass.
OUT=${OUT:-r05i}
export MICRO_GATHER_ONLY=lines
exec scripts/gpu_run.sh $OUT \
  time 120 tools/micro_gather :: \
  rdreq 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d gpurun_out/$OUT/rdreq -o p -- tools/micro_gather :: \
  fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/$OUT/fetch -o p -- tools/micro_gather :: \
  c3pmc 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d gpurun_out/$OUT/c3 -o p -- python3 tools/bench_paths.py --only c3
