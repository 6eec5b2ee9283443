#!/bin/bash
# Round 2: float64 arithmetic over float32-stored rows -- parity tests, then C3 bench legs
# per storage / compute dtype and the mixed-kernel A/B variants (DOPT_KRX_VARIANT).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale_parity.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r2_scale.log 2>&1 || { tail -30 gpurun_out/r2_scale.log; exit 1; }
tail -3 gpurun_out/r2_scale.log
B="python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --event-every 5"
timeout -k 10 240 $B --dtype float32 > gpurun_out/r2_b_f32.json 2> gpurun_out/r2_b_f32.err &&
timeout -k 10 240 $B --dtype float64 > gpurun_out/r2_b_f64.json 2> gpurun_out/r2_b_f64.err &&
timeout -k 10 240 $B --dtype float64 --data-dtype float32 > gpurun_out/r2_b_x32.json 2> gpurun_out/r2_b_x32.err &&
DOPT_KRX_VARIANT=14627 timeout -k 10 240 $B --dtype float64 --data-dtype float32 > gpurun_out/r2_b_x32_wide.json 2>&1 &&
DOPT_KRX_VARIANT=10243 timeout -k 10 240 $B --dtype float64 --data-dtype float32 > gpurun_out/r2_b_x32_plain.json 2>&1
rc=$?
for f in gpurun_out/r2_b_*.json; do echo "$f"; python -c "import json,sys; r=json.loads(open('$f').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r['roofline']['kernel_avg_ms'], r['final_objective'])" || tail -3 $f; done
exit $rc
