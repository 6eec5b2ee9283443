#!/bin/bash
# C5 row-space pass on one box: float32 engine (k_rs_pass<float>) vs float64 arithmetic over
# float32 rows (k_rs_pass_x32), alternated twice.
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 200 python -u tools/rs_ab.py --dtype float32 --reps 2 --shapes "2,6,2" > gpurun_out/ab_f32_$rep.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab_f32_$rep.log
  timeout -k 10 200 python -u tools/rs_ab.py --dtype float64 --data-dtype float32 --reps 2 --shapes "2,6,2" \
    > gpurun_out/ab_x32_$rep.log 2>&1 || exit 1
  tail -n 1 gpurun_out/ab_x32_$rep.log
done
