#!/bin/bash
# SQ counters of the C3 round kernel (one --pmc pass, SQ block only): wave cycles, waits, VALU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c3_sq
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/c3_sq -o run -- python -u bench.py --steps 10 --warmup 2 --no-secondary \
  --no-cpu-baseline > gpurun_out/c3_sq.log 2>&1 || { tail -n 20 gpurun_out/c3_sq.log; exit 1; }
python - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open("gpurun_out/c3_sq/run_counter_collection.csv")):
    acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "k_round" in k:
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVE_CYCLES", 1)
        print(k[:60], {c: round(x / w, 3) for c, x in m.items()})
PY
