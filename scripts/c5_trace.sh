#!/bin/bash
# C5 (quadratic, d = 2^20, complete graph) bench + kernel trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c5.log 2>&1 || exit $?
tail -n 1 gpurun_out/c5.log | cut -c 1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o run -- \
  python -u bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/c5prof.log 2>&1 || exit $?
python - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/c5prof/**/*kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:10.1f} us  {r["Percentage"]}%')
PY
