#!/bin/bash
# C5 shape: HBM bytes of the column-blocked step (separate FETCH_SIZE / WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/c5pmc
mkdir -p $OUT
export TMPDIR=/tmp
B="python -u bench.py --config c5 --steps 3 --warmup 0 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/hit -o run -- $B > $OUT/hit.log 2>&1 || exit $?
python - <<'PY'
import csv, glob, collections
for name in ("fetch", "write", "hit"):
    f = glob.glob(f"gpurun_out/c5pmc/{name}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(agg.items()):
        if "split" in k or "colsum" in k:
            print(f"{name:5s} {k:60s} {c:14s} n={len(v)} avg={sum(v)/len(v):.4g}")
PY
