#!/bin/bash
# Round-kernel time vs worker count (same work per worker): how much the last generation
# of workgroups (the kernel's tail) costs at C3's 4096.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WORKERS:-4096 8192 16384 2048}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --workers $w --steps 30 --event-every 1 > gpurun_out/w$w.log 2>&1 || exit 1
  python - "gpurun_out/w$w.log" $w <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r, w = d["roofline"], int(sys.argv[2])
print(w, "kernel %.4f ms" % r["kernel_avg_ms"], "TB/s %.3f" % (r["achieved"] / 1e3),
      "per-worker %.4f us" % (r["kernel_avg_ms"] * 1e3 / w), "ms/step %.4f" % d["ms_per_step"])
PY
done
