#!/bin/bash
# Round 5: K1 with the trimmed resolve rounds -- K1 parity tests, then the headline bench A/B/A/B
# against the previous build (reservoir_amd/libreservoir_hip_base.so)
OUT=${OUT:-r05tr3}
A="bench.py --no-secondary --no-cpu-baseline"
exec scripts/gpu_run.sh $OUT \
  test 400 python3 -u -m pytest tests/test_gpu_elements.py tests/test_gpu_configs.py tests/test_gpu_indexed.py -q -x --timeout 300 --timeout-method thread :: \
  base1 300 python3 tools/with_lib.py reservoir_amd/libreservoir_hip_base.so $A :: \
  new1 300 python3 $A :: \
  base2 300 python3 tools/with_lib.py reservoir_amd/libreservoir_hip_base.so $A :: \
  new2 300 python3 $A
