#!/bin/bash
# Round 6: the bucketed byte-key merge -- parity first, then the C4 UUID shares (A/B against the
# sort-based merge) and their timelines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06f}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide_distinct.py tests/test_gpu_wide_keys.py tests/test_gpu_distributed.py tests/test_gpu_ffm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  RSV_WIDE_BUCKETED=0 timeout -k 10 200 python3 tools/bench_paths.py --only c4w > $O/w_sort_$i.log 2>&1 || exit $?
  timeout -k 10 200 python3 tools/bench_paths.py --only c4w > $O/w_bucket_$i.log 2>&1 || exit $?
done
P="rocprofv3 --output-format csv --kernel-trace"
timeout -k 10 200 $P -d $O/ws -o ws -- python3 tools/bench_paths.py --only c4ws > $O/ws.log 2>&1 || exit $?
python3 tools/trace_window.py $O/ws/ws_kernel_trace.csv wide_filter_hashes 1 > $O/ws_timeline.txt || exit $?
timeout -k 10 200 $P -d $O/wu -o wu -- python3 tools/bench_paths.py --only c4wu > $O/wu.log 2>&1 || exit $?
python3 tools/trace_window.py $O/wu/wu_kernel_trace.csv wide_hash_all 1 > $O/wu_timeline.txt || exit $?
find $O -name "*_kernel_trace.csv" -delete
grep -h '^{' $O/w_*.log | cut -c1-250
echo done
