#!/bin/bash
# Round 2: in-process A/B of round-kernel variants on the C3 shape (tools/kr_variants.py).
# MODE f32 | x32 | f64, VARIANTS comma list (-1 = the default build).
set -o pipefail
mkdir -p gpurun_out
MODE=${MODE:-f64}
VARIANTS=${VARIANTS:--1,30755,145443,161827}
timeout -k 10 300 python -u tools/kr_variants.py --mode $MODE --reps 5 --rounds 10 \
  --variants=$VARIANTS > gpurun_out/r2_kr_ab_$MODE.json 2> gpurun_out/r2_kr_ab_$MODE.err
rc=$?
cat gpurun_out/r2_kr_ab_$MODE.json; tail -n 3 gpurun_out/r2_kr_ab_$MODE.err
exit $rc
