#!/bin/bash
# Round 5: the byte basis of random 8-B gathers (tools/micro_gather line probes): time, then the
# L2's memory-side read requests and FETCH_SIZE per probe, each counter set in its own pass; the
# packed-merge tests (rows snapshot, strict log retention); kernel stats of the wide C4 lines.
OUT=${OUT:-r05i}
P=/tmp/prof_$OUT
export MICRO_GATHER_ONLY=lines
exec scripts/gpu_run.sh $OUT \
  merge 300 python3 -u -m pytest tests/test_gpu_packed_merge.py -q -x --timeout 200 --timeout-method thread :: \
  time 120 tools/micro_gather :: \
  rdreq 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $P/rdreq -o p -- tools/micro_gather :: \
  fetch 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o p -- tools/micro_gather :: \
  c3pmc 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $P/c3 -o p -- python3 tools/bench_paths.py --only c3 :: \
  prof 300 rocprofv3 --kernel-trace --stats -d $P/stats -o w -- python3 tools/bench_paths.py --only c3k,c4w :: \
  copy 60 python3 tools/collect_small.py $P gpurun_out/$OUT
