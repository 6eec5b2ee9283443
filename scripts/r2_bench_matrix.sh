#!/bin/bash
# Round 2: bench.py option matrix on one GPU (each must print its JSON line), then the
# no-flag default run the driver's contract asks to finish within minutes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # run <name> <args...>
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bm_$name.json 2> gpurun_out/bm_$name.err || { echo "FAIL $name"; tail -n 20 gpurun_out/bm_$name.err; exit 1; }
  python - gpurun_out/bm_$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:10s} value {d['value']:.4g}  ms/step {d['ms_per_step']:.4f}  kernel {d['roofline']['kernel_avg_ms']:.4f} ms  frac {d['roofline']['frac']:.3f}  {d['roofline']['kernel'][:70]}")
PY
}
Q="--steps 20 --warmup 5 --no-cpu-baseline --no-secondary"
run b16 $Q --batch 16
run f32 $Q --dtype float32
run f64rows $Q --data-dtype float64
run pcie $Q --pcie
run phase16 $Q --phase --batch 16
run default
grep -o '"pcie": {[^}]*}' gpurun_out/bm_pcie.json | cut -c 1-300
