#!/bin/bash
# Round 6: the whole GPU suite, then K1's pooled tail A/B (tools/micro_k1o o), the C4 UUID shares
# (bucketed vs sort merge) with timelines, and one bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06i}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 tools/micro_k1o o 6144:10:2 6144:10:3 6144:9:3 5120:12:3 > $O/k1_tail.jsonl 2>&1 || { tail $O/k1_tail.jsonl; exit 1; }
grep tail $O/k1_tail.jsonl
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
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
echo done
