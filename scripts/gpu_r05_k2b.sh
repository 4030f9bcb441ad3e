#!/bin/bash
# Round 5: K2 with block FIFO entries -- A/B against the round-4 kernel (micro_k2 n), the segmented
# parity tests, the C3 line and a PMC VALU pass.
OUT=${OUT:-r05m}
P="rocprofv3 --output-format csv"
SQ="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  ab 300 tools/micro_k2 n :: \
  seg 600 python3 -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "segmented or c3 or ragged or fifo or long or pow27 or int32 or single" -x -q --timeout 300 --timeout-method thread :: \
  c3 200 python3 tools/bench_paths.py --only c3 :: \
  c3_sq 200 $P --pmc $SQ --kernel-trace -d $D/c3_sq -o pmc -- python3 tools/bench_paths.py --only c3 :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +4M -delete
