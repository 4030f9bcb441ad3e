#!/bin/bash
# Round-6 evidence run: smoke, the default bench line, rocprofv3 kernel stats + PMC passes for K1 (C2)
# and K2 (C3), K1's in-kernel clock, the secondary paths.  Summaries: tools/collect_profiles.py ->
# profiles/r06/ (pmc_summary.json)
OUT=${OUT:-r06z}
P="rocprofv3 --output-format csv"
SQ="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  suite 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  bench20 300 python3 bench.py --steps 20 --warmup 5 :: \
  bench 600 python3 bench.py :: \
  k1_trace 200 $P --kernel-trace --stats -d $D/k1 -o k1 -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary :: \
  k1_pmc_sq 120 $P --pmc $SQ --kernel-trace -d $D/k1_sq -o pmc -- $B :: \
  k1_pmc_fetch 120 $P --pmc FETCH_SIZE --kernel-trace -d $D/k1_fetch -o pmc -- $B :: \
  k1_pmc_write 120 $P --pmc WRITE_SIZE --kernel-trace -d $D/k1_write -o pmc -- $B :: \
  k1_clock 200 tools/micro_k1o k :: \
  c3_trace 200 $P --kernel-trace --stats -d $D/c3 -o c3 -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_sq 200 $P --pmc $SQ --kernel-trace -d $D/c3_sq -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  paths 400 python3 tools/bench_paths.py --only c4,c4r,c2i,c2h,c4m,c3k,c4w :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +4M -delete
