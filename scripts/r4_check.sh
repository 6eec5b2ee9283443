#!/bin/bash
# Round 4: the GPU tests most touched by this round's changes (parity incl. the trainers, the
# multi-GPU path, row-space subset), without stopping at the first failure, then the evidence of
# scripts/r4_c3_sq.sh (bench line, early-prologue A/B, strong-leg proxy, host probe).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== GPU tests"
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_distributed.py tests/test_gpu_rowspace.py -k "not test_rowspace_ or flag or ranks" \
  > gpurun_out/r4_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r4_tests.log | grep -v PASSED | head -30
tail -n 3 gpurun_out/r4_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # test failures: go on to the measurements; anything else: stop
bash scripts/r4_c3_sq.sh
