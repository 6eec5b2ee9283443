#!/bin/bash
# Round 4: the C5 row-space pass with one row group per column block (the new default) -- the
# row-space and full-size C5 tests, the 1 vs 2 row-group A/B (5 reps), the C5 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
echo "=== row-space tests"
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_rowspace.py \
  tests/test_gpu_fullsize.py tests/test_gpu_large_d.py -k "rowspace or c5" > gpurun_out/r4_c5c_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/r4_c5c_tests.log | head -20
tail -n 2 gpurun_out/r4_c5c_tests.log
[ $rc -eq 0 ] || exit $rc
echo "=== C5 row groups"
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 400 python3 tools/rs_ab.py --dtype float64 \
  --data-dtype float32 --reps 5 --shapes "2,8,1,1 2,8,2,1" > gpurun_out/r4_c5_groups.txt 2>&1 \
  || { tail -n 20 gpurun_out/r4_c5_groups.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_c5_groups.txt | tail -3
echo "=== C5 profile"
OUT=gpurun_out/prof_r4c5c PSTEPS=6 BENCH_ARGS="--config c5" bash scripts/profile.sh || exit 1
echo "=== done"
