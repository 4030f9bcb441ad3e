#!/bin/bash
# bench + rocprofv3 kernel-trace/stats summary (+ optional separate PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:---steps 10 --warmup 2}
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o k1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_$ctr -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$ctr.log 2>&1
    rc=$?; echo "pmc $ctr rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
if [ -n "$PMC" ]; then
  python tools/pmc_summary.py k1_resolve_publish 1000000000 gpurun_out/pmc_k1.json \
    gpurun_out/pmc_FETCH_SIZE/pmc_counter_collection.csv gpurun_out/pmc_WRITE_SIZE/pmc_counter_collection.csv
fi
find gpurun_out/prof -name "*.csv" 2>/dev/null || true
