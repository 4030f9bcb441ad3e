#!/bin/bash
# Round 5: the resolve stream (rsv_set_resolve_stream): its test, the headline bench A/B; the byte-
# basis PMC passes (csv) of the gather line probes and of K2; kernel stats of the large-k / wide lines.
OUT=${OUT:-r05j}
P="rocprofv3 --output-format csv"
S=/tmp/prof_$OUT
export MICRO_GATHER_ONLY=lines
exec scripts/gpu_run.sh $OUT \
  test 300 python3 -u -m pytest tests/test_gpu_resolve_stream.py tests/test_gpu_elements.py -q -x --timeout 200 --timeout-method thread :: \
  valu 120 tools/micro_valu :: \
  bench0 300 env RSV_BENCH_RESOLVE_STREAM=0 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench1 300 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench0b 300 env RSV_BENCH_RESOLVE_STREAM=0 python3 bench.py --no-secondary --no-cpu-baseline :: \
  bench1b 300 python3 bench.py --no-secondary --no-cpu-baseline :: \
  rdreq 120 $P --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $S/rdreq -o p -- tools/micro_gather :: \
  fetch 120 $P --pmc FETCH_SIZE --kernel-trace -d $S/fetch -o p -- tools/micro_gather :: \
  c3rdreq 200 $P --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d $S/c3 -o p -- python3 tools/bench_paths.py --only c3 :: \
  stats 300 $P --kernel-trace --stats -d $S/stats -o w -- python3 tools/bench_paths.py --only c3k,c4w :: \
  copy 60 python3 tools/collect_small.py $S gpurun_out/$OUT
