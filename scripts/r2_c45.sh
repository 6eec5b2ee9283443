#!/bin/bash
# Round 2: configs C4 and C5 at full size on one GPU -- the tests, then one bench line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 600 --timeout-method thread \
  > gpurun_out/r2_fullsize.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/r2_fullsize.log | tail -n 20; [ $rc -eq 0 ] || exit $rc
date +%s.%N > gpurun_out/t0; timeout -k 10 400 python -u bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/r2_c4.json 2> gpurun_out/r2_c4.err || { tail -n 30 gpurun_out/r2_c4.err; exit 1; }
tail -n 1 gpurun_out/r2_c4.json
timeout -k 10 400 python -u bench.py --config c5 --dtype float32 --steps 5 --warmup 2 > gpurun_out/r2_c5.json 2> gpurun_out/r2_c5.err || { tail -n 30 gpurun_out/r2_c5.err; exit 1; }
tail -n 1 gpurun_out/r2_c5.json
