#!/bin/bash
# Round 6: timelines of one UUID DISTINCT share (set mode / ordered mode): where the host waits
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
P="rocprofv3 --output-format csv --kernel-trace"
timeout -k 10 200 $P -d $O/ws -o ws -- python3 tools/bench_paths.py --only c4ws > $O/ws.log 2>&1 || exit $?
python3 tools/trace_window.py $O/ws/ws_kernel_trace.csv wide_filter_hashes 2 > $O/ws_timeline.txt || exit $?
timeout -k 10 200 $P -d $O/wu -o wu -- python3 tools/bench_paths.py --only c4wu > $O/wu.log 2>&1 || exit $?
python3 tools/trace_window.py $O/wu/wu_kernel_trace.csv wide_hash_all 2 > $O/wu_timeline.txt || exit $?
find $O -name "*_kernel_trace.csv" -delete
echo done
