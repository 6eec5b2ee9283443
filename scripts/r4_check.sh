#!/bin/bash
# Round 4: the multi-GPU path's GPU tests (lagged schedule with the sums in the exchange), then the
# baseline / counter / A/B / strong-proxy evidence of scripts/r4_c3_sq.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "=== distributed GPU tests"
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  tests/test_gpu_rowspace.py -k "not test_rowspace_ or flag or ranks" > gpurun_out/r4_dist_tests.log 2>&1; rc=$?
tail -n 25 gpurun_out/r4_dist_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/r4_c3_sq.sh
