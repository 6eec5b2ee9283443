#!/bin/bash
# Round 4: C5 pass, 4 KiB column blocks (half the row-dot partials) vs the default 2 KiB, both with
# every lane's row partial through LDS, one row group (A/B library, 5 reps interleaved).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 400 python3 tools/rs_ab.py --dtype float64 \
  --data-dtype float32 --reps 5 --shapes "4,4,1,1 2,8,1,1" > gpurun_out/r4_c5_cb4.txt 2>&1 \
  || { tail -n 20 gpurun_out/r4_c5_cb4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_c5_cb4.txt | tail -2
