#!/bin/bash
# Round 4: filter streaming shape A/B (dev builds): loads in flight per lane (U), workgroups per CU,
# candidate hashes recomputed on the rare slow path; C4 end to end (identity / set / ordered) each.
OUT=${OUT:-r04q}
W="python3 tools/with_lib.py"
exec scripts/gpu_run.sh $OUT \
  base 200 python3 tools/bench_paths.py --only c4 :: \
  g64 200 $W reservoir_amd/libreservoir_hip_expg64.so tools/bench_paths.py --only c4 :: \
  u16r 200 $W reservoir_amd/libreservoir_hip_expu16r.so tools/bench_paths.py --only c4 :: \
  u8r 200 $W reservoir_amd/libreservoir_hip_expu8r.so tools/bench_paths.py --only c4 :: \
  u16rg64 200 $W reservoir_amd/libreservoir_hip_expu16rg64.so tools/bench_paths.py --only c4 :: \
  base2 200 python3 tools/bench_paths.py --only c4
