#!/bin/bash
# development (round 2): K1 zero-mask queue v2 -- A/B, PMC, element tests, bench
D=gpurun_out/r02y
scripts/gpu_run.sh r02y k1ab 120 tools/micro_k1 a :: \
  k1pmc 120 rocprofv3 --output-format csv --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d $D/k1 -o pmc -- tools/micro_k1 p :: \
  tests 600 python -u -m pytest tests/test_gpu_elements.py tests/test_gpu_configs.py tests/test_gpu_cpp.py -m gpu -x -q -rfE --timeout 200 --timeout-method thread :: \
  bench 300 python3 bench.py --steps 50 --warmup 5 --no-secondary --no-cpu-baseline
