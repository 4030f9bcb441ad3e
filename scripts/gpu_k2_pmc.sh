#!/bin/bash
# K2 forms under one PMC pass (tools/micro_k2 l: wave-per-stream then lane-per-stream)
OUT=${OUT:-r02j}
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  k2_pmc 120 rocprofv3 --output-format csv --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $D/k2 -o pmc -- tools/micro_k2 l
