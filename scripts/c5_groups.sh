#!/bin/bash
# C5 column-blocked step time vs workgroups per launch (DOPT_SPLIT_WGS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in ${WGS:-4096 8192 16384 2048}; do
  DOPT_SPLIT_WGS=$g timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --event-every 1 > gpurun_out/c5g$g.log 2>&1 || exit 1
  python - "gpurun_out/c5g$g.log" $g <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("wgs", sys.argv[2], "step kernel %.3f ms" % d["roofline"]["kernel_avg_ms"], "TB/s %.3f" % (d["roofline"]["achieved"] / 1e3),
      "ms/round %.3f" % d["ms_per_step"])
PY
done
