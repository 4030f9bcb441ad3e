#!/bin/bash
# Round 4: HBM bytes of the C4 filters from PMC (FETCH_SIZE / WRITE_SIZE passes, one each):
# the ordered scheduled pass (sched_filter, c4o) and the set-mode filter (k3_filter, c4i).
OUT=${OUT:-r04c4p}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  c4o_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/c4_fetch -o pmc -- python3 tools/bench_paths.py --only c4o :: \
  c4o_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/c4_write -o pmc -- python3 tools/bench_paths.py --only c4o :: \
  c4i_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/c4i_fetch -o pmc -- python3 tools/bench_paths.py --only c4i :: \
  c4i_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/c4i_write -o pmc -- python3 tools/bench_paths.py --only c4i :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +4M -delete
