#!/bin/bash
# Round 4: the C5 row-space pass with the row dots through LDS after one DPP lane-pair add (LDOT 2,
# two workgroups per CU) vs every lane's partial through LDS (1) vs the DPP butterfly (0), A/B
# library, interleaved; then scripts/r4_full.sh (every GPU test, smoke, the default bench line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== C5 pass: LDOT 2 / 1 / 0"
DOPT_LIB=$PWD/distributed-optimization_amd/libdopt_ab.so timeout -k 10 300 python3 tools/rs_ab.py --dtype float64 \
  --data-dtype float32 --reps 3 --shapes "2,8,2,2 2,8,2,1 2,8,2,0" > gpurun_out/r4_c5_ldot2.txt 2>&1 \
  || { tail -n 20 gpurun_out/r4_c5_ldot2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4_c5_ldot2.txt
bash scripts/r4_full.sh
