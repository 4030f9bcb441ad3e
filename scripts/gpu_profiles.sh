#!/bin/bash
# Round profile set (one gpurun call): the default bench line, rocprofv3 kernel-trace/stats of the
# headline (K1) and of the C4 distinct path, and separate PMC passes (FETCH_SIZE, WRITE_SIZE) for
# K1 and the K3 filter.  Everything lands in gpurun_out/prof_r01/; the summaries worth keeping are
# copied into profiles/r01/ afterwards.  Every GPU step has its own time limit and the script
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/prof_r01
rm -rf "$O"
mkdir -p "$O"
step() {  # name, limit, command...
    local name=$1 limit=$2
    shift 2
    timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    [ $rc -eq 0 ] || { tail -20 "$O/$name.log"; exit $rc; }
}
step bench 400 python bench.py
tail -1 "$O/bench.log" > "$O/bench.json"
step k1_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/k1" -o k1 -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary
step c4_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c4" -o c4 -- \
    python3 tools/bench_paths.py --only c4i
for ctr in FETCH_SIZE WRITE_SIZE; do
    step "pmc_k1_$ctr" 180 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_k1_$ctr" -o pmc -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
    step "pmc_c4_$ctr" 180 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_c4_$ctr" -o pmc -- \
        python3 tools/bench_paths.py --only c4i
done
f() { find "$O/$1" -name "*counter_collection.csv" | head -1; }
python tools/pmc_summary.py k1_resolve_publish 1000000000 "$O/pmc_k1.json" "$(f pmc_k1_FETCH_SIZE)" "$(f pmc_k1_WRITE_SIZE)"
python tools/pmc_summary.py k3_filter 500000000 "$O/pmc_k3.json" "$(f pmc_c4_FETCH_SIZE)" "$(f pmc_c4_WRITE_SIZE)"
find "$O" -name "*stats.csv"
