#!/bin/bash
# Round 4, second pass: the multi-GPU GPU tests (incl. the complete graph as CSR rows longer than
# k_mixcs's register-held entries, and the C2 trainers at 2 ranks), then scripts/r4_sq.sh (SQ
# counters, C5 row-dot A/B, PMC profiles).  Test failures go on to the measurements; a crash,
# abort or time limit stops here.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== multi-GPU tests"
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  > gpurun_out/r4_dist2.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_dist2.log | grep -v PASSED | head -30
tail -n 3 gpurun_out/r4_dist2.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r4_sq.sh
