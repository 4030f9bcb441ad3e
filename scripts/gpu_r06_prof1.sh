#!/bin/bash
# Round 6: where the byte-key DISTINCT share spends its time (rocprof kernel stats, set and ordered
# mode), what K1's timing events cost the 20-step headline (--time-every 6 vs 2, A/B/A/B), and K1's
# in-kernel clock (tools/micro_k1o k: stamped diagnostic copy) for the PMC normalisation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
P="rocprofv3 --output-format csv --kernel-trace --stats"
timeout -k 10 120 tools/micro_k1o k > $O/k1clk.log 2>&1 || exit $?
timeout -k 10 200 $P -d $O/ws -o ws -- python3 tools/bench_paths.py --only c4ws > $O/ws.log 2>&1 || exit $?
timeout -k 10 200 $P -d $O/wu -o wu -- python3 tools/bench_paths.py --only c4wu > $O/wu.log 2>&1 || exit $?
for i in 1 2; do
  for te in 6 2; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --time-every $te > $O/b_te${te}_$i.json 2>$O/b_te${te}_$i.err || exit $?
  done
done
find $O -name "*_kernel_trace.csv" -size +4M -delete
echo done
