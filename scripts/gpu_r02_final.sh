#!/bin/bash
# Round-2 closing run (one gpurun call): the GPU suite and smoke, the default bench line, and the
# rocprofv3 evidence behind its roofline figures -- kernel stats + PMC passes for K1 (the C2 bench)
# and K2 (C3), and the C3 winner-gather floor (tools/micro_gather).  Output: gpurun_out/$OUT/
# (summaries copied into profiles/r02/ by tools/collect_profiles.py).
OUT=${OUT:-r02f}
P="rocprofv3 --output-format csv"
SQ="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  pytest 700 python3 -u -m pytest tests -m gpu -q -rfE -x --timeout 300 --timeout-method thread :: \
  smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" :: \
  bench 500 python3 bench.py --steps 50 --warmup 5 :: \
  k1_trace 200 $P --kernel-trace --stats -d $D/k1 -o k1 -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary :: \
  k1_pmc_sq 120 $P --pmc $SQ --kernel-trace -d $D/k1_sq -o pmc -- $B :: \
  k1_pmc_fetch 120 $P --pmc FETCH_SIZE --kernel-trace -d $D/k1_fetch -o pmc -- $B :: \
  k1_pmc_write 120 $P --pmc WRITE_SIZE --kernel-trace -d $D/k1_write -o pmc -- $B :: \
  c3_trace 200 $P --kernel-trace --stats -d $D/c3 -o c3 -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_sq 200 $P --pmc $SQ --kernel-trace -d $D/c3_sq -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_fetch 200 $P --pmc FETCH_SIZE --kernel-trace -d $D/c3_fetch -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  c3_pmc_write 200 $P --pmc WRITE_SIZE --kernel-trace -d $D/c3_write -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  gather_trace 120 $P --kernel-trace --stats -d $D/gather -o gather -- tools/micro_gather :: \
  gather_pmc_fetch 120 $P --pmc FETCH_SIZE --kernel-trace -d $D/gather_fetch -o pmc -- tools/micro_gather :: \
  c4_trace 200 $P --kernel-trace --stats -d $D/c4 -o c4 -- python3 tools/bench_paths.py --only c4o
