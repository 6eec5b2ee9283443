#!/bin/bash
# Round 2: in-process A/B of the float64-over-float32-rows round kernel variants (C3 shape),
# then the float32 kernel with deferred loss terms / xbar in LDS.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kr_variants.py --mode x32 --reps 5 --rounds 10 \
  --variants=-1,161827,751651,751907 > gpurun_out/r2_krx_ab.json 2> gpurun_out/r2_krx_ab.err &&
timeout -k 10 300 python -u tools/kr_variants.py --mode f32 --reps 5 --rounds 10 \
  --variants=-1,145699 > gpurun_out/r2_kr_ab.json 2> gpurun_out/r2_kr_ab.err
rc=$?
cat gpurun_out/r2_krx_ab.json gpurun_out/r2_kr_ab.json; tail -n 3 gpurun_out/r2_krx_ab.err; tail -n 3 gpurun_out/r2_kr_ab.err
exit $rc
