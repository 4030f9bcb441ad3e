#!/bin/bash
# Round 6: where the Long hash-twin replay's time goes (RSV_REPLAY_DEBUG: per segment to-host and run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r06r}
mkdir -p $O
RSV_REPLAY_DEBUG=1 timeout -k 10 300 python3 tools/bench_paths.py --only c4r > $O/c4r.log 2>&1 || { tail -20 $O/c4r.log; exit 1; }
grep -h "rsv replay\|^{" $O/c4r.log | tail -20 | cut -c1-300
echo done
