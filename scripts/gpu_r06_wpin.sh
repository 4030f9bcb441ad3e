#!/bin/bash
# Round 6: the byte-key replay from persistent pinned copies (one wait for log + flags) -- parity of
# the wide distinct tests (twins at full size, export_log, multi-rank UUID) and the UUID twin share
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06p}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide_distinct.py tests/test_gpu_wide_keys.py tests/test_gpu_distributed.py tests/test_gpu_ffm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  RSV_REPLAY_DEBUG=1 timeout -k 10 300 python3 tools/bench_paths.py --only c4w > $O/c4w_$i.log 2>&1 || exit 1
done
grep -h "wide replay" $O/c4w_*.log | tail -4
grep -h '^{' $O/c4w_*.log | python3 -c "import json,sys; [print(json.loads(l)['config'][60:140], json.loads(l)['seconds_end_to_end']) for l in sys.stdin]"
echo done
