#!/bin/bash
# Row-space rounds: the GPU tests (incl. multi-rank), then the pass-shape A/B at C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rowspace.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/rs_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/rs_tests.log | tail -n 30; exit 1; }
grep -E "passed|failed" gpurun_out/rs_tests.log | tail -n 2
timeout -k 10 700 python -u tools/rs_ab.py ${RS_AB_ARGS:-} > gpurun_out/rs_ab.log 2>&1 || { tail -n 20 gpurun_out/rs_ab.log; exit 1; }
tail -n 8 gpurun_out/rs_ab.log
