#!/bin/bash
# Round-2 profile set (one gpurun call): VALU issue costs + clock (PMC on tools/micro_valu), the
# default bench line, rocprofv3 kernel stats and PMC passes for K1 (C2 bench) and K2 (C3).
# Output: gpurun_out/$OUT/ (summaries get copied into profiles/r02/).
OUT=${OUT:-r02z}
P="rocprofv3 --output-format csv"
SQ="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  valu_pmc 90 $P --pmc $SQ --kernel-trace -d $D/valu_pmc -o pmc -- tools/micro_valu :: \
  bench 500 python3 bench.py --steps 50 --warmup 5 :: \
  k1_trace 200 $P --kernel-trace --stats -d $D/k1 -o k1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary :: \
  k1_pmc_sq 120 $P --pmc $SQ --kernel-trace -d $D/k1_sq -o pmc -- $B :: \
  k1_pmc_fetch 120 $P --pmc FETCH_SIZE --kernel-trace -d $D/k1_fetch -o pmc -- $B :: \
  k1_pmc_write 120 $P --pmc WRITE_SIZE --kernel-trace -d $D/k1_write -o pmc -- $B :: \
  c3_trace 200 $P --kernel-trace --stats -d $D/c3 -o c3 -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_sq 200 $P --pmc $SQ --kernel-trace -d $D/c3_sq -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/c3_fetch -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/c3_write -o pmc -- python3 tools/bench_paths.py --only c3
