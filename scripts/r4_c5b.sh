#!/bin/bash
# Round 4: C5 pass shapes with every lane's row partial through LDS (LDOT 1): 8 vs 16 rows in flight
# per wave, 1 / 2 / 4 row groups (A/B library, interleaved), then the C5 profile (kernel stats +
# FETCH_SIZE / WRITE_SIZE passes) of the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
echo "=== C5 pass shapes"
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 400 python3 tools/rs_ab.py --dtype float64 \
  --data-dtype float32 --reps 3 --shapes "2,8,2,1 2,16,2,1 2,8,4,1 2,8,1,1" > gpurun_out/r4_c5_shapes.txt 2>&1 \
  || { tail -n 20 gpurun_out/r4_c5_shapes.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_c5_shapes.txt
echo "=== C5 profile (x32 row-space rounds)"
OUT=gpurun_out/prof_r4c5b PSTEPS=6 BENCH_ARGS="--config c5" bash scripts/profile.sh || exit 1
echo "=== done"
