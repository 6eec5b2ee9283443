#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ramp
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ramp -o run -- python -u tools/ramp_probe.py \
  > gpurun_out/ramp.log 2>&1 || { tail -n 20 gpurun_out/ramp.log; exit 1; }
python - <<'PY'
import csv
rows = [r for r in csv.DictReader(open("gpurun_out/ramp/run_kernel_trace.csv")) if "k_round" in r["Kernel_Name"] and "true, true" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(len(d))
for k in range(0, len(d), 10):
    print(k, " ".join("%.3f" % x for x in d[k:k + 10]))
PY
