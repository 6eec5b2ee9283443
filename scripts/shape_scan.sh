#!/bin/bash
# Round-kernel bandwidth at equal bytes per launch but different workgroup sizes:
# workers x rows pairs (PAIRS="4096:512 8192:256 16384:128"), full-shard batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in ${PAIRS:-4096:512 8192:256 16384:128 2048:1024}; do
  w=${p%%:*}; m=${p##*:}
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --workers $w --m $m --steps 30 --event-every 1 > gpurun_out/s$w.log 2>&1 || exit 1
  python - "gpurun_out/s$w.log" $w $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "x", sys.argv[3], "kernel %.4f ms" % r["kernel_avg_ms"], "TB/s %.3f" % (r["achieved"] / 1e3),
      "ms/step %.4f" % d["ms_per_step"])
PY
done
