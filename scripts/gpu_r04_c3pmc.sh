#!/bin/bash
# Round 4: HBM bytes of K2 (C3) and of the plain winner-key gather at the same shape (its floor,
# tools/micro_gather) from PMC (FETCH_SIZE / WRITE_SIZE passes, one each).
OUT=${OUT:-r04c3p}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  c3_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/c3_fetch -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  c3_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/c3_write -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  g_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/gather_fetch -o pmc -- ./tools/micro_gather :: \
  g_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/gather_write -o pmc -- ./tools/micro_gather :: \
  g_time 100 ./tools/micro_gather :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +4M -delete
