#!/bin/bash
# Row-space C5 rounds: GPU tests (small cases vs the oracle / direct rounds, C5 at full size),
# then the C5 bench line with the row-space rounds and with the direct ones (DOPT_ROWSPACE=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rowspace.py tests/test_gpu_large_d.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/rs_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/rs_tests.log | tail -n 30; exit 1; }
grep -E "passed|failed" gpurun_out/rs_tests.log | tail -n 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k c5 -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/rs_full.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert" gpurun_out/rs_full.log | tail -n 30; exit 1; }
grep -E "passed|failed" gpurun_out/rs_full.log | tail -n 2
timeout -k 10 300 python -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/rs_c5.json 2> gpurun_out/rs_c5.err || { tail -n 20 gpurun_out/rs_c5.err; exit 1; }
tail -n 1 gpurun_out/rs_c5.json | cut -c 1-1500
DOPT_ROWSPACE=0 timeout -k 10 300 python -u bench.py --config c5 --dtype float32 --steps 20 --warmup 3 --no-cpu-baseline \
  > gpurun_out/rs_c5_direct.json 2> gpurun_out/rs_c5_direct.err || { tail -n 20 gpurun_out/rs_c5_direct.err; exit 1; }
tail -n 1 gpurun_out/rs_c5_direct.json | cut -c 1-600
echo "=== done"
