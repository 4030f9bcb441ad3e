#!/bin/bash
# Round 6: Philox scalar-operand trims + full-round zm assumption (product) vs the previous code
# (libreservoir_hip_expold.so, -DRSV_R6_OLD): parity subset, then C2 bench and C3 A/B/A/B, PMC VALU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06t}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_elements.py tests/test_gpu_segmented.py tests/test_gpu_configs.py -k "c1 or c2 or c3 or segmented or ragged or elements" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OLD=reservoir_amd/libreservoir_hip_expold.so
B="bench.py --no-cpu-baseline --no-secondary"
for i in 1 2; do
  timeout -k 10 200 python3 tools/with_lib.py $OLD $B > $O/b_old_$i.json 2> $O/b_old_$i.err || { tail $O/b_old_$i.err; exit 1; }
  timeout -k 10 200 python3 $B > $O/b_new_$i.json 2> $O/b_new_$i.err || { tail $O/b_new_$i.err; exit 1; }
done
for f in $O/b_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], r['launch_avg_us'], r['frac'], r.get('launches_timed'))"; done
for i in 1 2; do
  timeout -k 10 200 python3 tools/with_lib.py $OLD tools/bench_paths.py --only c3 > $O/c3_old_$i.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/bench_paths.py --only c3 > $O/c3_new_$i.log 2>&1 || exit 1
done
grep -h -o '"seconds": [0-9.]*' $O/c3_*.log
P="rocprofv3 --output-format csv"
SQ="SQ_INSTS_VALU SQ_WAVE_CYCLES"
timeout -s KILL 120 $P --pmc $SQ --kernel-trace -d $O/new_sq -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $O/new_sq.log 2>&1 || exit 1
timeout -s KILL 120 $P --pmc $SQ --kernel-trace -d $O/old_sq -o pmc -- python3 tools/with_lib.py $OLD bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary > $O/old_sq.log 2>&1 || exit 1
timeout -s KILL 120 $P --pmc $SQ --kernel-trace -d $O/c3new_sq -o pmc -- python3 tools/bench_paths.py --only c3 > $O/c3new_sq.log 2>&1 || exit 1
timeout -s KILL 120 $P --pmc $SQ --kernel-trace -d $O/c3old_sq -o pmc -- python3 tools/with_lib.py $OLD tools/bench_paths.py --only c3 > $O/c3old_sq.log 2>&1 || exit 1
python3 tools/pmc_kernels.py $O/new_sq $O/new_sq.json k1_last_writer | tail -3
python3 tools/pmc_kernels.py $O/old_sq $O/old_sq.json k1_last_writer | tail -3
python3 tools/pmc_kernels.py $O/c3new_sq $O/c3new_sq.json k2_segmented | tail -3
python3 tools/pmc_kernels.py $O/c3old_sq $O/c3old_sq.json k2_segmented | tail -3
find $O -name "*_kernel_trace.csv" -delete
echo done
