#!/bin/bash
# One gpurun session: GPU tests, smoke, bench.  Each GPU step has its own time limit; a crash
# (exit status other than 0/1) stops the script before any further GPU step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-tests -m gpu -q -rfE}
BENCH_ARGS=${BENCH_ARGS:---steps 10 --warmup 2}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
