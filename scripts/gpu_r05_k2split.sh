#!/bin/bash
# Round 5: VALU split of K2 at C3's shape from the cost-probe variants (tools/micro_k2 c / g under PMC)
OUT=${OUT:-r05t}
P="rocprofv3 --output-format csv"
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  c 300 $P --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $D/c -o c -- tools/micro_k2 c :: \
  g 300 $P --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $D/g -o g -- tools/micro_k2 g :: \
  trim 30 find $D -name "*_kernel_trace.csv" -size +4M -delete
