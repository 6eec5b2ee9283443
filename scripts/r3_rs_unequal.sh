#!/bin/bash
# Row-space rounds from unequal starting iterates: the row-space test file, then the C5 x32 line
# from a random start (bench --c5-start random) beside the zero start.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_rowspace.py tests/test_gpu_large_d.py tests/test_gpu_checkpoint.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rsu_tests.log 2>&1
rc=$?; grep -E "FAIL|Error|error|passed|failed" gpurun_out/rsu_tests.log | tail -n 12; [ $rc -eq 0 ] || exit $rc
