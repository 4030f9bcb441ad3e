#!/bin/bash
# Round 6: K1's final resolve rounds pooled per workgroup in the SECOND group only (its four waves
# start and end together) vs per-wave tails everywhere (tools/micro_k1o o: per_wave_tail vs pooled_tail)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r06w}
mkdir -p $O
timeout -k 10 300 tools/micro_k1o o 6144:10:2 6144:10:3 6144:10:4 > $O/k1_hyb.jsonl 2>&1 || { tail $O/k1_hyb.jsonl; exit 1; }
grep tail $O/k1_hyb.jsonl
echo done
