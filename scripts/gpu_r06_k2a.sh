#!/bin/bash
# Round 6: K2 append loop with a running LDS address -- parity (segmented + C3) and C3 VALU / time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06u}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "segmented or ragged or c3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python3 tools/bench_paths.py --only c3 > $O/c3_$i.log 2>&1 || exit 1
done
grep -h -o '"seconds": [0-9.]*' $O/c3_*.log
timeout -s KILL 120 rocprofv3 --output-format csv --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $O/c3_sq -o pmc -- python3 tools/bench_paths.py --only c3 > $O/c3_sq.log 2>&1 || exit 1
python3 tools/pmc_kernels.py $O/c3_sq $O/c3_sq.json k2_segmented | grep '"SQ_INSTS_VALU"'
find $O -name "*_kernel_trace.csv" -delete
echo done
