#!/bin/bash
# Round time vs HIP-event sampling period (1 = every launch, 10 = bench default, 0 = none).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in a b; do
  for e in 1 10 0; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --event-every $e ${BENCH_ARGS:-} > gpurun_out/ev$e$rep.log 2>&1 || exit $?
    python - "gpurun_out/ev$e$rep.log" "every=$e rep=$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel", r["kernel_avg_ms"],
      "launches", r["kernel_launches_timed"], "frac", r["frac"])
PY
  done
done
