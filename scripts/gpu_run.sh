#!/bin/bash
# gpurun helper: run named steps, each under its own time limit, stop at the first failure.
#   scripts/gpu_run.sh <outdir> <name> <limit> <command...> [:: <name> <limit> <command...>]...
# (steps are separated by "::" -- "--" is left alone for rocprofv3's program separator)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
while [ $# -gt 0 ]; do
    name=$1 limit=$2
    shift 2
    cmd=()
    while [ $# -gt 0 ] && [ "$1" != "::" ]; do cmd+=("$1"); shift; done
    [ "$1" == "::" ] && shift
    echo "== $name (limit $limit s): ${cmd[*]}"
    timeout -k 10 "$limit" "${cmd[@]}" > "$O/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc"
    tail -n 12 "$O/$name.log"
    [ $rc -eq 0 ] || exit $rc
done
