#!/bin/bash
# C5 row-space rounds with float32-stored rows under float64 arithmetic (k_rs_pass_x32):
# parity tests, the pass-shape A/B, and the bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rowspace.py tests/test_gpu_large_d.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/x32_tests.log 2>&1 || { tail -n 40 gpurun_out/x32_tests.log; exit 1; }
tail -n 3 gpurun_out/x32_tests.log
timeout -k 10 300 python -u tools/rs_ab.py --dtype float64 --data-dtype float32 --reps 2 \
  --shapes "2,6,2 2,4,2 2,3,2 1,8,2 4,2,2" > gpurun_out/x32_ab.log 2>&1 || { tail -n 20 gpurun_out/x32_ab.log; exit 1; }
tail -n 6 gpurun_out/x32_ab.log
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/x32_bench.log 2>gpurun_out/x32_bench.err \
  || { tail -n 20 gpurun_out/x32_bench.err; exit 1; }
cat gpurun_out/x32_bench.log
