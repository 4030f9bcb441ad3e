#!/bin/bash
# Round 6: the ordered replay with the next segment staged on the device while the host replays the
# current one -- parity (ordered replay tests, the full-size twin configs, the multi-rank replays)
# and the C4 Long / UUID twin shares with RSV_REPLAY_OVERLAP=0 / 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06o}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distinct.py tests/test_gpu_configs.py tests/test_gpu_distributed.py tests/test_gpu_packed_merge.py -k "ordered or replay or c4 or twin or distributed or log" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  RSV_REPLAY_OVERLAP=0 RSV_REPLAY_DEBUG=1 timeout -k 10 300 python3 tools/bench_paths.py --only c4r > $O/c4r_off_$i.log 2>&1 || exit 1
  RSV_REPLAY_DEBUG=1 timeout -k 10 300 python3 tools/bench_paths.py --only c4r > $O/c4r_on_$i.log 2>&1 || exit 1
done
for f in $O/c4r_*.log; do echo $f; grep -h "rsv replay" $f | tail -3; grep -h '^{' $f | python3 -c "import json,sys; [print(json.loads(l)['seconds_end_to_end']) for l in sys.stdin]"; done
echo done
