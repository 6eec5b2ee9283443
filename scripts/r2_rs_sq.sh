#!/bin/bash
# SQ counters of the C5 row-space pass (one --pmc pass, SQ block only): wave cycles, waits, VALU.
# ENGINE="--dtype float32" (default) or "--dtype float64" (float32 rows, k_rs_pass_x32); TAG names the output.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ENGINE=${ENGINE:---dtype float32}
TAG=${TAG:-rs_sq}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/$TAG -o run -- python -u bench.py --config c5 $ENGINE --steps 4 --warmup 1 \
  --no-cpu-baseline > gpurun_out/$TAG.log 2>&1 || { tail -n 20 gpurun_out/$TAG.log; exit 1; }
TAG=$TAG python - <<'PY'
import csv, collections, os
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f"gpurun_out/{os.environ['TAG']}/run_counter_collection.csv")):
    acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "rs_pass" in k or "split_step" in k:
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVE_CYCLES", 1)
        print(k[:60], {c: round(x / w, 3) for c, x in m.items()})
PY
