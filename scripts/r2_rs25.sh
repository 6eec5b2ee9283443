#!/bin/bash
# Row-space pass shape 2 / 5 (x32: 224 VGPRs, 2 waves per SIMD) vs 2 / 6 (260 registers, 1 wave),
# both engines, interleaved in one process each.
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rs_ab.py --dtype float64 --data-dtype float32 --reps 3 --shapes "2,6,2 2,5,2" \
  > gpurun_out/rs25_x32.log 2>&1 || { tail -n 20 gpurun_out/rs25_x32.log; exit 1; }
tail -n 2 gpurun_out/rs25_x32.log
timeout -k 10 300 python -u tools/rs_ab.py --dtype float32 --reps 3 --shapes "2,6,2 2,5,2" \
  > gpurun_out/rs25_f32.log 2>&1 || { tail -n 20 gpurun_out/rs25_f32.log; exit 1; }
tail -n 2 gpurun_out/rs25_f32.log
