#!/bin/bash
# C3 round-kernel durations launch by launch (kernel trace of a 60-round bench run): the
# even / odd alternation of the fused round kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/alt -o run -- \
  python3 -u bench.py --no-cpu-baseline --no-secondary --steps ${STEPS:-60} --warmup 5 ${BENCH_ARGS:-} > gpurun_out/alt.log 2>&1 \
  || { tail -n 20 gpurun_out/alt.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/alt/**/run_kernel_trace.csv", recursive=True) + glob.glob("gpurun_out/alt/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
d = [(e - s) / 1e3 for s, e, n in ks if "k_round<" in n and "true, true" in n]
print(len(d), "launches:", " ".join("%.0f" % x for x in d))
ev, od = d[0::2], d[1::2]
print("even mean %.1f  odd mean %.1f" % (sum(ev) / len(ev), sum(od) / len(od)))
PY
