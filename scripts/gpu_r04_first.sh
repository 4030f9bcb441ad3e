#!/bin/bash
# Round 4: replay through first-occurrence flags -- distinct + config parity, the replay line,
# a fresh ordered-distinct kernel timeline (tools/timeline.py).
OUT=${OUT:-r04fo}
D=gpurun_out/$OUT
exec scripts/gpu_run.sh $OUT \
  dist 600 python3 -u -m pytest tests/test_gpu_distinct.py -q -rfE -x --timeout 300 --timeout-method thread :: \
  twins 300 env RSV_REPLAY_DEBUG=1 python3 tools/bench_paths.py --only c4r :: \
  c4tl 200 rocprofv3 --output-format csv --kernel-trace -d $D/c4 -o c4 -- python3 tools/bench_paths.py --only c4o
