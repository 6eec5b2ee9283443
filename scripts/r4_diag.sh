#!/bin/bash
# Round 4: the C2 trainers at 1 and 2 gloo ranks vs the reference fixture (every label), then the
# measurements of scripts/r4_c3_sq.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== trainer diagnostic"
timeout -k 10 300 python3 tools/diag_trainers2.py > gpurun_out/r4_diag.log 2>&1; rc=$?
grep -v "amdgpu.ids\|socket.cpp\|Gloo\|Spectral\|Running\|finished" gpurun_out/r4_diag.log | head -60
[ $rc -eq 0 ] || exit $rc
bash scripts/r4_c3_sq.sh
